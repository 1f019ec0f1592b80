"""Probe: the multi-rank render paths (parallel.py) over RCCL ("nccl") with every rank on
cuda:0 of a one-GPU box.  Usage: python tools/rccl_probe.py WORLD.  Prints one JSON line
per path with the max abs difference to the single-launch render."""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from mpi_vision_amd import _host, _lib, configs, parallel
    H, W, P, V = 37, 53, 11, 5
    mpi = configs.synthetic_mpi(1, H, W, P, 5)
    K = configs.f32([configs.intrinsics_matrix(50.0, 52.0, 26.0, 18.0)] * V)
    poses = configs.f32([configs.pose_from(configs.rot_y(1.5 - v), (0.05 * v, -0.02, 0.03)) for v in range(V)])
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 20, P)), K, V).to(dev)
    packed = _lib.pack_planes(mpi[0].to(dev))
    frames = parallel.render_view_sharded(packed, homs, gather=True)
    p0, p1 = parallel.shard_range(P, rank, world)
    local = _lib.pack_planes(mpi[0, :, :, p0:p1].contiguous().to(dev))
    frame = parallel.render_plane_sharded(local, homs[:1, p0:p1].contiguous(), H)
    if rank == 0:
        seq = _lib.render_packed(packed, homs)
        res = {"world": world, "backend": dist.get_backend(),
               "view_sharded_bit_exact": bool(torch.equal(frames, seq)),
               "plane_sharded_max_abs": float((frame - seq[:1]).abs().max())}
        with open(out, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1])
    out = os.path.join(REPO, "gpurun_out", f"rccl_probe_w{world}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
    with open(out) as f:
        print(f.read())

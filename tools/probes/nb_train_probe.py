"""Where the notebook-shape training step's 0.19 ms goes (224x224, 10 planes, bs 1): host time
of each Python-level piece (perf_counter, no synchronisation) vs the device span of n steps.
Probe only (GPU box): python tools/probes/nb_train_probe.py > gpurun_out/nb_probe.json"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

dev = torch.device("cuda:0")
N, P, n = 224, 10, 200
depths = mv.inv_depths(1, 100, P)
f = configs.focal_from_fov(N)
K = configs.f32(configs.intrinsics_matrix(f, f, N / 2.0, N / 2.0)).to(dev)[None]
pose = configs.f32(configs.pose_from(configs.rot_y(1.0), (0.05, -0.02, 0.03))).to(dev)[None]
planes = configs.f32(depths).to(dev)
mpi = configs.synthetic_mpi(1, N, N, P, 9).to(dev)
leaf = mpi.clone().requires_grad_(True)
g = torch.Generator(device=dev).manual_seed(5)
dout = torch.rand((1, N, N, 3), generator=g, device=dev)


def host_us(fn, k=n):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        fn()
    h = (time.perf_counter() - t) / k * 1e6
    torch.cuda.synchronize()
    return h


def dev_us(fn, k=n):
    for _ in range(20):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(k):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / k * 1e3


def step():
    o = mv.mpi_render_view_torch(leaf, pose, planes, K)
    o.backward(dout)
    leaf.grad = None


homs = _host.render_homographies_device(pose, planes, K, 1)
out, ck = _lib.render_train(leaf.detach(), homs)
ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(N, N, P), dtype=torch.uint8, device=dev)
res = {
    "step_span_us": dev_us(step), "step_host_us": host_us(step),
    "homs_host_us": host_us(lambda: _host.render_homographies_device(pose, planes, K, 1)),
    "fwd_dropin_nograd_host_us": host_us(lambda: mv.mpi_render_view_torch(mpi, pose, planes, K)),
    "render_train_host_us": host_us(lambda: _lib.render_train(leaf.detach(), homs)),
    "render_train_dev_us": dev_us(lambda: _lib.render_train(leaf.detach(), homs)),
    "bwd_host_us": host_us(lambda: _lib.render_backward(leaf.detach(), homs, dout, ckpt=ck)),
    "bwd_ws_host_us": host_us(lambda: _lib.render_backward(leaf.detach(), homs, dout, workspace=ws, ckpt=ck)),
    "bwd_dev_us": dev_us(lambda: _lib.render_backward(leaf.detach(), homs, dout, workspace=ws, ckpt=ck)),
    "bwd_nocheck_dev_us": dev_us(lambda: _lib.render_backward(leaf.detach(), homs, dout, workspace=ws, ckpt=ck,
                                                             check=False)),
    "empty_call_host_us": host_us(lambda: _lib._call("mpiv_mark", 1, _lib._stream(dev))),
    "empty_call_dev_us": dev_us(lambda: _lib._call("mpiv_mark", 1, _lib._stream(dev))),
}
print(json.dumps({k: round(v, 2) for k, v in res.items()}))

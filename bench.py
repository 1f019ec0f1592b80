#!/usr/bin/env python3
"""Headline benchmark: rendered Mpix/s of the fused MPI warp + over-composite on
BASELINE.json config 4 (128-plane 1024x1024 MPI, 1000-pose camera path,
view-sharded), with the dominant kernel's roofline and the CPU restatement timed on
the same host, plus a config-5 leg (256-plane 4096x2160 MPI, plane-sharded).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--views V] [--no-config5]

One process per GPU (torchrun for N > 1).  Each rank holds a full MPI replica in
HBM (packed plane-major once, outside the timed region) and every step renders
V views of the camera path (rank r renders path poses r*V .. r*V+V-1 modulo the
path), so per-GPU work is fixed as N grows ("weak"); at N = 8 and V = 125 one step
is exactly the 1000-pose path.  There is no collective on the data path.

Per step (inside the timed region): host-side homographies for the NEXT step
(torch-CPU fp32, the reference's op order) overlap the current launch; then one
render launch writes V frames [V,1024,1024,3] fp32 that stay in HBM.

Roofline.  The V views of one launch share one MPI, so the texels
they gather come from L2 (hit rate ~0.99): what bounds the kernel is the vector-memory
("texture") path that serves the gathers, not HBM.  `roofline` therefore prices the
launch against that path: bytes = the 16-B gather instructions the launch issues x 1 KiB
(four per plane-sample for the direct kernel; fewer with the rows kernel's vertical tap
reuse, counted live by its census build), peak = the gather rate the same device reaches
with the render's access shape (mpiv_probe_gather, measured live).  HBM is reported separately, with fractions
that cannot exceed 1: `hbm_traffic_frac` (PMC bytes actually moved per launch, from the
committed rocprofv3 summary of this same command, only if its build id / kernel / shape
match) and `single_view` (one view per launch: every texel is read once, so its
algorithmic bytes P*H*W*16 + H*W*12 really cross HBM -- the north-star 0.60 bar).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from mpi_vision_amd import _host, _lib, configs, parallel  # noqa: E402

METRIC = "rendered Mpix/sec (node) + achieved HBM GB/s fraction, 1024²×128-plane MPI"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
kWaveBytes = 64 * 16   # one 64-lane 16-B gather instruction


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--views", type=int, default=125, help="views rendered per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget (0 = skip)")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 plane-sharded leg")
    ap.add_argument("--no-training", action="store_true",
                    help="skip the training (render backward) leg: its gated cooperative fallback launch makes "
                         "rocprofv3 --kernel-trace crash in its own teardown (DESIGN.md section 7)")
    ap.add_argument("--no-extras", action="store_true",
                    help="only the timed config-4 launches (rocprofv3 runs: tools/profile.sh), no frame check, "
                         "single-view leg, gather probe or config-5 leg")
    ap.add_argument("--kernel", choices=["packed", "packed_mv", "packed_lds", "native"], default="packed",
                    help="packed: direct-gather kernel on the packed MPI (default); packed_mv: multi-view "
                         "LDS kernel (A/B); packed_lds: single-view LDS variant (A/B); native: reference "
                         "layout read in place")
    return ap.parse_args()


def dist_setup(args):
    """One process per GPU (torchrun env).  MPIV_BENCH_BACKEND=gloo + MPIV_BENCH_ONE_DEVICE=1
    rehearse the multi-rank logic on a single-GPU box (all ranks on cuda:0, CPU collectives)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if os.environ.get("MPIV_BENCH_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        import torch.distributed as dist
        backend = os.environ.get("MPIV_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, torch.device("cuda", local)


def max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def load_pmc(profile_dir: str, kernel: str, views: int, shape):
    """The committed rocprofv3 PMC summary of this bench command (tools/profile.sh ->
    tools/parse_pmc.py -> profiles/render_pmc.json), or None unless it was taken from the
    same library build (source hash), kernel, views per launch and MPI shape."""
    path = os.path.join(profile_dir, "render_pmc.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    want = {"build_id": _lib.load().mpiv_build_id().decode(), "kernel": kernel, "views": views,
            "shape": list(shape)}
    if any(d.get(k) != v for k, v in want.items()):
        return None
    return d


def event_ms(fn, n, stream):
    """Average device time of fn() over n calls, HIP events on the launch stream."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def gather_peak_gbs(dev, stream):
    """The texture path's gather ceiling on this device (mpiv_probe_gather: 16-B-per-lane
    buffer loads with the render's access shape from an L1/L2-resident window)."""
    window = torch.zeros(4096, device=dev)
    sink = torch.zeros(4, device=dev)
    blocks, iters = 2048, 2048
    fn = lambda: _lib._call("mpiv_probe_gather", window, iters, blocks, sink, _lib._stream(dev))  # noqa: E731
    fn()
    ms = event_ms(fn, 5, stream)
    return blocks * 256 * iters * 128 / (ms * 1e-3) / 1e9


def cpu_baseline(mpi_dev: torch.Tensor, homs_all: torch.Tensor, budget_s: float, check_frames):
    """The oracle's C restatement (bit-exact to the reference) on this host's cores,
    on a bounded sample: whole views of the same MPI, as many as fit ~budget_s."""
    from oracle import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    mpi = mpi_dev.cpu().numpy()[None]          # [1,H,W,P,4]
    H, W = mpi.shape[1], mpi.shape[2]
    views, t_total, outs = 0, 0.0, []
    while views == 0 or (t_total < budget_s and views < homs_all.shape[0]):
        h = homs_all[views:views + 1].numpy()
        t0 = time.perf_counter()
        o = oracle.render(mpi, h, threads)
        t_total += time.perf_counter() - t0
        outs.append(o)
        views += 1
    mism = 0
    for i, o in enumerate(outs[:len(check_frames)]):
        if not np.array_equal(o, check_frames[i]):
            mism += 1
    return {"value": views * H * W / 1e6 / t_total, "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{views} full view(s) of the 1024x1024x128 MPI with the oracle's C restatement "
                      f"(oracle/mpiv_oracle.c, {threads} OpenMP threads), {t_total:.1f} s",
            "gpu_frames_bit_exact_vs_cpu": mism == 0}


def sha16(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]


def training_leg(dev, stream, n=10):
    """The training caller's path at config-4 size (notebook loss, ipynb cell 12 L42: a
    non-broadcast [1,H,W,P,4] MPI rendered and differentiated): the training forward
    (frame + composite checkpoints, mpiv_render_train) and the bit-exact backward
    (mpiv_render_backward) fed those checkpoints, plus the backward without them; HIP
    events on the launch stream, one view, synthetic data generated on the device."""
    c4 = configs.config4()
    H, W, P = c4["H"], c4["W"], c4["P"]
    g = torch.Generator(device=dev).manual_seed(7)
    mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c4["poses"][100:101]), configs.f32(c4["depths"]),
                                     configs.f32([c4["K"]]), 1).to(dev)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    fwd_ms = event_ms(lambda: _lib.render_train(mpi, homs), n, stream)
    g1 = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
    bwd_ms = event_ms(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck), n, stream)
    g2 = _lib.render_backward(mpi, homs, dout, workspace=ws)
    bwd2_ms = event_ms(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws), n, stream)
    flag = int(ws[_lib.bwd_flag_offset(H, W, P):][:4].view(torch.int32).item())
    same = bool(torch.equal(g1.view(torch.int32), g2.view(torch.int32)))
    mpi_bytes = P * H * W * 16
    res = {"workload": "BASELINE config 4 MPI (1024x1024x128), one non-broadcast view: training forward + backward",
           "forward_ms": round(fwd_ms, 4), "backward_ms": round(bwd_ms, 4),
           "backward_no_ckpt_ms": round(bwd2_ms, 4), "step_ms": round(fwd_ms + bwd_ms, 4),
           "backward_alg_bytes": 2 * mpi_bytes + H * W * 12,
           "backward_alg_def": "MPI read + d MPI written + d frame read (workspace traffic not counted)",
           "backward_hbm_frac": round((2 * mpi_bytes + H * W * 12) / (bwd_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "workspace_GB": round(ws.numel() / 1e9, 3), "fallback_flag": flag,
           "ckpt_grad_bit_identical": same}
    del mpi, ws, g1, g2, ck
    torch.cuda.empty_cache()
    return res


def config5_leg(world, rank, dev, steps, warmup):
    """BASELINE config 5: the 256-plane 4096x2160 MPI (36.2 GB), one pose, planes sharded
    over the ranks.  Each rank generates its plane range on the device (counter-based
    synth.hip, outside the timed region).  Step at N = 1: one render of all 256 planes;
    at N > 1: render_plane_sharded -- the rank's (C, T) partial, one all-to-all of row
    bands (RCCL point-to-point over xGMI), the ordered combine of its band, and the gather
    of the RGB bands to rank 0.  Total work is fixed ("strong" scaling)."""
    c = configs.config5()
    H, W, P = c["H"], c["W"], c["P"]
    homs = _host.render_homographies(configs.f32(c["poses"]), configs.f32(c["depths"]), configs.f32([c["K"]]), 1)
    p0, p1 = parallel.shard_range(P, rank, world)
    hl = homs[:, p0:p1].contiguous().to(dev)
    stream = torch.cuda.current_stream(dev)
    packed = _lib.synth_mpi_packed(c["seed"], H, W, p0, p1, dev)
    if world == 1:
        out = torch.empty((1, H, W, 3), device=dev)
        launch = lambda: _lib._call("mpiv_render_packed", packed, H, W, p1 - p0, hl, 1, out,  # noqa: E731
                                    _lib._stream(dev))

        def step():
            launch()
            return out
        shard_bytes = P * H * W * 16 + H * W * 12
    else:
        ct = torch.empty((1, H, W, 4), device=dev)
        launch = lambda: _lib._call("mpiv_render_packed_ct", packed, H, W, p1 - p0, 0, p1 - p0,  # noqa: E731
                                    int(rank == 0), hl, 1, ct, _lib._stream(dev))
        step = lambda: parallel.render_plane_sharded(packed, hl, H)  # noqa: E731
        shard_bytes = (p1 - p0) * H * W * 16 + H * W * 16
    kern_ms = event_ms(launch, 3, stream)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        frame = step()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    kern_ms = max_over_ranks(kern_ms, world, dev)
    res = {"workload": "BASELINE config 5: 256-plane 4096x2160 MPI (36.2 GB), 1 pose, plane-sharded",
           "value": round(steps * H * W / 1e6 / elapsed, 2), "unit": "Mpix/s", "n_gpus": world,
           "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "scaling": "strong",
           "data": "synthetic (counter-based per-shard generator, synth.hip, seed 0)",
           "planes_per_gpu": p1 - p0, "shard_kernel_ms": round(kern_ms, 3),
           "shard_alg_bytes": shard_bytes,
           "shard_hbm_frac": round(shard_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "parallelism": "single GPU, sequential render" if world == 1 else
           f"plane-sharded x{world}: (C,T) partials + band all-to-all + ordered combine + gather",
           "frame_sha16": sha16(frame) if rank == 0 else None}
    del packed
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if args.kernel == "packed_mv":
        _lib.load().mpiv_debug_set(b"render_mv", 1)  # libmpiv's debug option (A/B)
    world, rank, dev = dist_setup(args)
    torch.cuda.set_device(dev)
    c4 = configs.config4()
    H, W, P = c4["H"], c4["W"], c4["P"]
    V = args.views
    n_path = len(c4["poses"])

    def make_view():
        gen = torch.Generator(device=dev).manual_seed(c4["seed"])
        v = torch.rand((H, W, P, 4), generator=gen, device=dev, dtype=torch.float32)
        v[..., :3].mul_(2.0).sub_(1.0)
        v[:, :, 0, 3] = 1.0
        return v

    # --- resident inputs: one MPI replica per GPU (generated on device), packed once
    view = make_view()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    packed = _lib.pack_planes(view) if args.kernel.startswith("packed") else None
    # mpiv_render_packed's routing (abi.hip render_packed_impl): a near-square MPI at 1-2 or
    # >= 32 views per launch goes to the R-rows-per-lane kernel, other view counts gather
    # one row per work-item
    rows = abs(W / (H - 1) - 1.0) <= 0.25 and (V <= 2 or V >= 32)
    kernel_name = {"packed": "render_rows_kernel" if rows else "render_packed_kernel",
                   "packed_lds": "render_lds_kernel", "native": "render_chunk_kernel",
                   "packed_mv": "render_mv_kernel" if V >= 4 else "render_packed_kernel"}[args.kernel]
    entry = "mpiv_render_packed_lds" if args.kernel == "packed_lds" else "mpiv_render_packed"
    torch.cuda.synchronize()
    pack_ms = (time.perf_counter() - t0) * 1e3

    poses = configs.f32(c4["poses"])
    K = configs.f32(c4["K"])
    depths = configs.f32(c4["depths"])

    def step_indices(s):
        base = (rank * V + s * world * V) % n_path
        return [(base + j) % n_path for j in range(V)]

    def host_homs(s, n=V):
        idx = step_indices(s)[:n]
        return _host.render_homographies(poses[idx], depths, K.expand(n, 3, 3), n)

    out = torch.empty((V, H, W, 3), device=dev, dtype=torch.float32)
    hbuf = [torch.empty((V, P, 9), dtype=torch.float32).pin_memory() for _ in range(2)]
    dbuf = [torch.empty((V, P, 9), device=dev, dtype=torch.float32) for _ in range(2)]
    stream = torch.cuda.current_stream(dev)

    def launch(h_dev, n, o):
        if packed is not None:
            _lib._call(entry, packed, H, W, P, h_dev, n, o, _lib._stream(dev))
        else:
            mpi5 = view.unsqueeze(0).expand(n, H, W, P, 4)
            _lib._call("mpiv_render", mpi5, _lib._strides(mpi5), n, H, W, P, h_dev, o, _lib._stream(dev))

    copied = [None, None]  # event recorded after the last H2D copy out of each pinned slot

    def upload(s):
        slot = s % 2
        if copied[slot] is not None:
            copied[slot].synchronize()  # the DMA has read this pinned buffer; safe to refill
        hbuf[slot].copy_(host_homs(s))
        dbuf[slot].copy_(hbuf[slot], non_blocking=True)  # stream-ordered after earlier launches
        ev = torch.cuda.Event()
        ev.record(stream)
        copied[slot] = ev

    def run(n_steps, first, events=None):
        upload(first)
        for s in range(first, first + n_steps):
            if events is not None:
                events[s - first][0].record(stream)
            launch(dbuf[s % 2], V, out)
            if events is not None:
                events[s - first][1].record(stream)
            if s + 1 < first + n_steps:
                upload(s + 1)  # host-side homographies of the next step overlap this launch

    # single-view leg (one view per launch: every texel crosses HBM once, the north-star
    # 0.60 bar), measured before the sustained multi-view load so it does not inherit a
    # lowered clock from it
    one = torch.empty((1, H, W, 3), device=dev)
    sv_ms = float("nan")
    if not args.no_extras:
        h_sv = host_homs(0, 1).to(dev)
        for _ in range(50):  # ~25 ms of untimed launches: the clocks leave their idle state first
            launch(h_sv, 1, one)
        sv_ms = event_ms(lambda: launch(h_sv, 1, one), 20, stream)

    run(args.warmup, 0)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    t0 = time.perf_counter()
    run(args.steps, args.warmup, events)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, world, dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))

    # --- after the timed region: the last timed launch's first frame against a one-view
    # launch of the same pose (bit-exact), the single-view leg, the gather ceiling
    last = args.warmup + args.steps - 1
    timed_frame_sha = one_sha = None
    peak_gbs = float("nan")
    gathers = None
    if not args.no_extras:
        timed_frame_sha = sha16(out[0])
        h1 = host_homs(last, 1).to(dev)
        launch(h1, 1, one)
        torch.cuda.synchronize()
        one_sha = sha16(one[0])
        peak_gbs = gather_peak_gbs(dev, stream)
        # the texture path's real work in the timed launches: the counting build of the same
        # kernel (mpiv_render_packed_census) re-renders the timed steps and adds up the
        # 64-lane 16-B gather instructions its waves issue (vertical tap reuse gathers fewer
        # than the four taps per plane-sample of the direct kernel)
        if packed is not None and entry == "mpiv_render_packed":
            census = torch.zeros(1, dtype=torch.int64, device=dev)
            try:  # every timed step's views (the count depends on the poses), averaged per launch
                for s_ in range(args.warmup, args.warmup + args.steps):
                    _lib._call("mpiv_render_packed_census", packed, H, W, P, host_homs(s_).to(dev), V, out, census,
                               _lib._stream(dev))
                gathers = int(census.item()) // args.steps
            except RuntimeError:  # this view count does not route to the rows kernel
                gathers = None

    mpix_total = world * args.steps * V * H * W / 1e6
    value = mpix_total / elapsed
    tap_bytes = V * P * H * W * 64            # four 16-B taps per plane-sample (direct kernel)
    hbm_alg_bytes = V * (P * H * W * 16 + H * W * 12)  # every view reading its MPI once (§8d)
    sv_bytes = P * H * W * 16 + H * W * 12
    gather_bytes = gathers * kWaveBytes if gathers else tap_bytes  # what the texture path moves
    achieved = gather_bytes / (kern_ms * 1e-3) / 1e9
    pmc = load_pmc(os.path.join(REPO, "profiles"), kernel_name, V, (H, W, P))
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None

    del out
    if packed is not None:
        del view
    torch.cuda.empty_cache()
    train = training_leg(dev, stream) if (world == 1 and not args.no_extras and not args.no_training) else None
    c5 = None if (args.no_config5 or args.no_extras) else config5_leg(world, rank, dev, max(3, args.steps // 2), 1)

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded U[-1,1) rgb / U[0,1) alpha MPI generated on device; viewer-style 1000-pose sway path)",
            "config": {"workload": "BASELINE config 4: 128-plane 1024x1024 MPI, 1000-pose camera path, view-sharded",
                       "H": H, "W": W, "planes": P, "views_per_gpu_per_step": V, "kernel": args.kernel,
                       "parallelism": f"view-sharded x{world} (replicas, no data-path collective)",
                       "views_per_s": round(value / (H * W / 1e6), 2), "pack_ms_once": round(pack_ms, 2)},
            "roofline": {
                "bound": "texture", "achieved": round(achieved, 1),
                "peak": round(peak_gbs, 1) if peak_gbs == peak_gbs else None, "unit": "GB/s",
                "frac": round(achieved / peak_gbs, 4) if peak_gbs == peak_gbs else None, "traffic": traffic,
                "kernel": kernel_name, "kernel_ms_per_launch": round(kern_ms, 3),
                "alg_bytes_per_launch": gather_bytes,
                "alg_bytes_def": ("gather instructions the launch issues (counted live by the kernel's census build, "
                                  "mpiv_render_packed_census) x 64 lanes x 16 B" if gathers else
                                  "V*P*H*W*64: four 16-B bilinear taps per plane-sample through the vector-memory path"),
                "gathers_per_plane_sample": round(gathers * 64 / (V * P * H * W), 3) if gathers else 4.0,
                "alg_bytes_4tap": tap_bytes,
                "peak_def": "mpiv_probe_gather on this device: 16-B/lane buffer loads, render access shape, "
                            "L1/L2-resident window (MI355X_MICROARCH.md L2: 34.5-36.9 TB/s)",
                "ta_busy_frac": pmc.get("ta_busy_frac") if pmc else None,
                "l2_hit_rate": pmc.get("l2_hit_rate") if pmc else None,
                "hbm_traffic_frac": round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "mpi_reuse_per_launch": round(hbm_alg_bytes / traffic, 1) if traffic else None,
                "single_view": None if args.no_extras else {
                    "kernel_ms": round(sv_ms, 4), "alg_bytes": sv_bytes,
                    "achieved_gbs": round(sv_bytes / (sv_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                    "frac": round(sv_bytes / (sv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bound": "hbm"},
                "pmc_source": "profiles/render_pmc.json (same build id / kernel / views / shape)" if pmc else
                              "no matching profiles/render_pmc.json for this build",
            },
            "timed_frame_check": {"frame": "view 0 of the last timed launch vs a 1-view launch of its pose",
                                  "sha16": timed_frame_sha, "bit_exact": timed_frame_sha == one_sha},
            "cpu_baseline": None,
            "config5_plane_sharded": c5,
            "training_render_backward": train,
        }
        if world == 1 and args.cpu_seconds > 0 and not args.no_extras:
            # the GPU frame of the first view of step 0, to cross-check the CPU sample bit-exactly
            hs = host_homs(0)
            launch(hs[:1].to(dev), 1, one)
            torch.cuda.synchronize()
            res["cpu_baseline"] = cpu_baseline(make_view(), hs, args.cpu_seconds, [one.cpu().numpy()])
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

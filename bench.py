#!/usr/bin/env python3
"""Headline benchmark: rendered Mpix/s of the fused MPI warp + over-composite on
BASELINE.json config 4 (128-plane 1024x1024 MPI, 1000-pose camera path,
view-sharded), with the dominant kernel's roofline and the CPU restatement timed on
the same host, plus one leg per other BASELINE config and the notebook's own shape.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--views V] [--legs c4,sv,...]

Launch.  One process per GPU.  `--gpus N > 1` without a torchrun environment starts
N ranks itself (a `torch.distributed.run` child, before this process touches the GPU)
and exits with its status; with WORLD_SIZE set (the driver's own torchrun launch) it
must equal --gpus.  Ranks talk over RCCL ("nccl"); MPIV_BENCH_BACKEND=gloo +
MPIV_BENCH_ONE_DEVICE=1 rehearse the multi-rank logic on a one-GPU box.

Headline (config 4, "weak").  Each rank holds a full MPI replica in HBM (packed
plane-major once, outside the timed region) and every step renders V views of the
camera path (rank r renders path poses r*V .. r*V+V-1 modulo the path), so per-GPU
work is fixed as N grows; at N = 8 and V = 125 one step is exactly the 1000-pose path.
There is no collective on the data path.  Per step (inside the timed region):
host-side homographies for the NEXT step (the reference's torch-CPU fp32 op order)
overlap the current launch; then one render launch writes V frames [V,1024,1024,3]
fp32 that stay in HBM.

Roofline.  The V views of one launch share one MPI, so the texels
they gather come from L2: what bounds the launch is the vector-memory ("texture")
path that serves the gathers, not HBM.  `roofline` prices the launch against that
path: bytes = the 16-B gather instructions the launch issues x 1 KiB (counted live by
the kernel's census build), peak = the gather rate the same device reaches with the
render's access shape (mpiv_probe_gather, measured live: a TA ceiling, not a spec
peak).  HBM is reported per leg with fractions that cannot exceed 1: `single_view`
(one view per launch: every texel crosses HBM once, the north-star 0.60 bar), the
PSV (config 3) and the config-5 shard.

rocprofv3 evidence.  tools/profile.sh runs this script under rocprofv3 and
tools/parse_prof.py groups the dispatches by (kernel, grid size) into
profiles/prof_summary.json, tagged with the library build id.  Every leg names the
kernel and grid its launch routes to (mpiv_route) and, when the summary's build id
matches this library, quotes rocprof's average duration and the PMC HBM traffic of
exactly those dispatches next to its own HIP-event time.

Legs (--legs, default all): c4 (headline), sv (single view), c2 (config 2: 64 views
of a 1024x576x32 MPI), c3 (config 3: PSV of 5 sources into 64 planes through
plane_sweep_torch), nb (the notebook's 224x224x10 render + training step + PSV),
u8 (8-bit texels: config-4-shape u8 MPI, one view and V views per launch), netout (the
network output rendered in one kernel at config 2's size), train (config-4-size training
forward + backward), c5 (config 5, plane-sharded), cpu (the CPU baseline, rank 0 at N = 1).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
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
ALL_LEGS = ("c4", "sv", "c2", "c3", "nb", "u8", "netout", "train", "c5", "cpu")
# SURVEY.md §6 / BASELINE.md: the reference utils.py on torch-CPU (MKL), 8 Xeon cores,
# measured in the survey container (the reference cannot run on the GPU box)
REF_CPU = {"c4_Mpix_s": 0.37, "c4_s_per_view": 2.8727, "c3_s": 5.858, "c2_proxy_Mpix_s": 1.49,
           "cores": 8, "source": "SURVEY.md §6: reference utils.py on torch 2.10 CPU, 8 Xeon cores, survey container"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--views", type=int, default=125, help="views rendered per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget (0 = skip)")
    ap.add_argument("--legs", default=",".join(ALL_LEGS), help="comma list of " + ",".join(ALL_LEGS))
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 leg")
    ap.add_argument("--no-training", action="store_true", help="skip the training leg")
    ap.add_argument("--no-extras", action="store_true", help="only the timed config-4 launches")
    ap.add_argument("--kernel", choices=["packed", "native"], default="packed",
                    help="packed: the production packed-MPI route (default); native: the reference layout "
                         "read in place (mpiv_render)")
    a = ap.parse_args()
    legs = [x for x in a.legs.split(",") if x]
    bad = [x for x in legs if x not in ALL_LEGS]
    if bad:
        ap.error(f"unknown legs {bad}")
    if a.no_extras:
        legs = [x for x in legs if x == "c4"]
    if a.no_config5:
        legs = [x for x in legs if x != "c5"]
    if a.no_training:
        legs = [x for x in legs if x != "train"]
    if a.cpu_seconds <= 0:
        legs = [x for x in legs if x != "cpu"]
    a.legs = legs
    return a


def spawn_ranks(n: int) -> int:
    """--gpus N > 1 outside torchrun: run this script as N ranks under a
    torch.distributed.run child (127.0.0.1 rendezvous on a free port) and wait.  Called
    before anything touches the GPU; rank 0's JSON line reaches stdout directly."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


# Collective timeout of the bench's process group: well under the driver's 600-s limit for the whole
# run, and longer than LEG_DEADLINE_S, so a hung exchange is ended by the LineGuard (which still
# prints the line) before RCCL's watchdog would tear the process down without it.
PG_TIMEOUT_S = float(os.environ.get("MPIV_BENCH_PG_TIMEOUT", "150"))
# Wall-clock limit of the plane-sharded (config-5) leg at world > 1 -- the only leg with a data-path
# collective -- counted from its start to the end of the run.
LEG_DEADLINE_S = float(os.environ.get("MPIV_BENCH_LEG_DEADLINE", "90"))


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    local = 0 if os.environ.get("MPIV_BENCH_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    if world > 1:
        import datetime
        torch.cuda.set_device(local)
        import torch.distributed as dist
        backend = os.environ.get("MPIV_BENCH_BACKEND", "nccl")
        timeout = datetime.timedelta(seconds=PG_TIMEOUT_S)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    return world, rank, torch.device("cuda", local), backend


def max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks(x: float, world: int, dev) -> list:
    if world == 1:
        return [x]
    import torch.distributed as dist
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _json_scalar(o):
    """numpy scalars (and 0-d arrays) that reach the bench line serialise as Python numbers."""
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, np.ndarray) and o.ndim == 0:
        return o.item()
    raise TypeError(f"Object of type {type(o).__name__} is not JSON serializable")


class LineGuard:
    """Rank 0's one JSON line, printed exactly once, even when a collective leg hangs.

    The plane-sharded leg (config 5) is the only one with a data-path exchange, and the driver's
    8-GPU node is the first place it runs over RCCL at world > 1.  `guarded()` turns an exception
    into an error field, but a hang would keep rank 0 from ever printing the headline it has
    already measured.  So every rank arms a timer before that leg: if the leg (and the final
    barrier / process-group teardown after it) has not finished by the deadline, rank 0 prints
    the line with the leg's error field and every rank leaves with os._exit (an exit, not an
    exec: no new program starts in the GPU-initialised process)."""

    def __init__(self, rank: int, out=None):
        import threading
        self.rank = rank
        self.out = out or sys.stdout
        self.lock = threading.Lock()
        self.printed = False
        self.timer = None

    def emit(self, res: dict) -> bool:
        """Print res as the line (rank 0 only; at most once). True if this call printed it."""
        with self.lock:
            if self.rank != 0 or self.printed:
                return False
            self.printed = True
            self.out.write(json.dumps(res, default=_json_scalar) + "\n")
            self.out.flush()
            return True

    def arm(self, seconds: float, res: dict, leg: str):
        """From now on, `seconds` of wall clock until the run must have ended."""
        import threading

        def expire():
            res[leg] = {"error": f"timed out: the leg and the run's teardown did not finish within {seconds:.0f} s "
                                 "(a hung collective); the other legs' figures are complete"}
            self.emit(res)
            sys.stderr.write(f"bench.py rank {self.rank}: {leg} timed out after {seconds:.0f} s, exiting\n")
            sys.stderr.flush()
            os._exit(0)
        self.timer = threading.Timer(seconds, expire)
        self.timer.daemon = True
        self.timer.start()

    def disarm(self):
        if self.timer is not None:
            self.timer.cancel()
            self.timer = None


def fault_injected(name: str, rank: int) -> bool:
    """MPIV_BENCH_FAULT=<name>: rehearse a failure of the plane-sharded exchange on the last rank
    (c5_hang: it stops answering; c5_raise: it raises) -- tests of LineGuard / guarded only."""
    return os.environ.get("MPIV_BENCH_FAULT") == name and rank == int(os.environ.get("WORLD_SIZE", "1")) - 1


# ---------------------------------------------------------------------------
# rocprofv3 evidence (tools/profile.sh -> tools/parse_prof.py)
# ---------------------------------------------------------------------------

_PROF = None


def prof_summary():
    """profiles/prof_summary.json when it was taken from this library build, else None."""
    global _PROF
    if _PROF is None:
        path = os.path.join(REPO, "profiles", "prof_summary.json")
        _PROF = {}
        if os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            if d.get("build_id") == _lib.load().mpiv_build_id().decode():
                _PROF = d
    return _PROF or None


def prof_for(kernel: str, grid: int, tag: str | None = None):
    """The summary's entry for the dispatches of `kernel` with `grid` work-items inside the timed
    region marked `tag` (mpiv_mark phase tags), or over the whole run (tag None or no tagged entry)."""
    d = prof_summary()
    if not d:
        return None
    whole = None
    for e in d.get("launches", []):
        if e["kernel"] == kernel and e["grid"] == grid:
            if tag is not None and e.get("tag") == tag:
                return e
            if "tag" not in e:
                whole = e
    return whole


def prof_tag_kernels(tag: str, calls_per_region: int):
    """Every libmpiv kernel the summary saw inside the region marked `tag`, by total time: per
    kernel the rocprof average, dispatches per call of the region's operation and the PMC HBM
    traffic per dispatch (the backward's chain, gather, ... separately)."""
    d = prof_summary()
    if not d:
        return None
    out = []
    for e in d.get("launches", []):
        if e.get("tag") == tag and e.get("calls"):
            out.append({"kernel": e["kernel"], "grid_workitems": e["grid"], "rocprof_avg_ms": round(e["avg_ns"] / 1e6, 4),
                        "dispatches_per_call": round(e["calls"] / calls_per_region, 2),
                        "ms_per_call": round(e["avg_ns"] / 1e6 * e["calls"] / calls_per_region, 4),
                        "traffic": e.get("hbm_bytes"), "valu_issue_frac": e.get("valu_issue_frac"),
                        "ta_busy_frac": e.get("ta_busy_frac")})
    return sorted(out, key=lambda x: -x["ms_per_call"])


def mark(name: str, dev):
    """Phase marker (mpiv_mark) for the rocprof summary: the dispatches after it belong to `name`."""
    _lib._call("mpiv_mark", configs.PROF_TAGS[name], _lib._stream(dev))


def prof_fields(kernel: str, grid: int, alg_bytes: float, ms: float, tag: str | None = None):
    """rocprof average and PMC traffic of this leg's launch, with the ratios the verdict
    recomputes: rocprof ms vs the bench's own HIP-event ms, HBM traffic vs algorithmic bytes.
    tag: the leg's timed region (its dispatches only, when the summary has them)."""
    e = prof_for(kernel, grid, tag)
    res = {"kernel": kernel, "grid_workitems": grid,
           "prof_source": "profiles/prof_summary.json (same build id)" if e else "no rocprof summary of this build"}
    if e:
        res["prof_region"] = e.get("tag", "all dispatches of this kernel and grid")
        res["rocprof_avg_ms"] = round(e["avg_ns"] / 1e6, 4)
        res["rocprof_calls"] = e["calls"]
        # the summary comes from another run (tools/profile.sh): a leg whose rocprof average is
        # more than 5 % away from this run's event time is flagged, not silently quoted
        res["rocprof_over_event"] = round(e["avg_ns"] / 1e6 / ms, 3)
        res["rocprof_agrees_5pct"] = abs(e["avg_ns"] / 1e6 / ms - 1.0) <= 0.05
        if e.get("hbm_bytes") is not None:
            res["traffic"] = e["hbm_bytes"]
            res["traffic_over_alg"] = round(e["hbm_bytes"] / alg_bytes, 3)
            res["traffic_frac"] = round(e["hbm_bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        for k in ("fetch_kib", "write_kib", "l2_hit_rate", "ta_busy_frac", "valu_issue_frac"):
            if e.get(k) is not None:
                res[k] = e[k]
    return res


# ---------------------------------------------------------------------------
# timing helpers
# ---------------------------------------------------------------------------

# Device time of untimed launches before each timed region.  After a host-side gap (an allocation,
# a check with a host sync) the next ~25 ms of launches run up to 40 % slower on the box before they
# settle (config 3: 0.88 vs 0.61 ms per launch; profiles/r05_c3_ramp.jsonl), so a few untimed
# launches are not a warm-up; every leg now runs >= WARM_MS of back-to-back launches first.
WARM_MS = 60.0


def warm(fn, stream, min_ms=WARM_MS, cap=5000):
    """Untimed back-to-back calls of fn for about min_ms of device time (the count from 2 timed
    calls, then enqueued without a host sync); returns the number of calls."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    fn()
    fn()
    b.record(stream)
    b.synchronize()
    per = max(a.elapsed_time(b) / 2, 1e-3)
    k = min(cap, int(np.ceil(min_ms / per)))
    for _ in range(k):
        fn()
    return k + 2


def event_ms(fn, n, stream, each=False):
    """Average device time of fn() over n calls, HIP events on the launch stream (each: the list)."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in ev]
    return t if each else float(np.mean(t))


def span_ms(fn, n, stream):
    """Device time of n back-to-back calls / n (host work between launches overlaps)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(n):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def gather_peak_gbs(dev, stream):
    """The texture path's gather ceiling on this device (mpiv_probe_gather: 16-B-per-lane
    buffer loads with the render's access shape from an L1/L2-resident window)."""
    window = torch.zeros(4096, device=dev)
    sink = torch.zeros(4, device=dev)
    blocks, iters = 2048, 2048
    fn = lambda: _lib._call("mpiv_probe_gather", window, window.numel() * 4, iters, blocks, sink,  # noqa: E731
                            _lib._stream(dev))
    fn()
    ms = event_ms(fn, 5, stream)
    return blocks * 256 * iters * 128 / (ms * 1e-3) / 1e9


def sha16(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]


def gen_view(H, W, P, seed, dev):
    """Synthetic MPI view [H,W,P,4] on the device: rgb U[-1,1), alpha U[0,1), plane-0 alpha 1."""
    gen = torch.Generator(device=dev).manual_seed(seed)
    v = torch.rand((H, W, P, 4), generator=gen, device=dev, dtype=torch.float32)
    v[..., :3].mul_(2.0).sub_(1.0)
    v[:, :, 0, 3] = 1.0
    return v


def hbm(alg_bytes, ms):
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    return round(gbs, 1), round(gbs / HBM_PEAK_GBS, 4)


def sampled_boxes(homs: np.ndarray, H: int, W: int) -> np.ndarray:
    """Texel boxes [V, P, 4] (x0, x1, y0, y1, inclusive, clamped to the image) that the
    reference's render samples for each (view, plane).  The sample position of output pixel
    (x, y) is linear-fractional in (x, y) (utils.py:186-188: u/w, v/w, then the SWAPPED
    normalisation x/(H-1), y/(W-1) and grid_sample's unnormalise), so while w keeps its sign
    over the frame its extremes lie at the 4 frame corners; a plane whose w changes sign gets
    the whole image.  The bilinear taps add one texel right and below."""
    h = homs.reshape(homs.shape[0], -1, 3, 3).astype(np.float64)
    xs = np.array([0.0, W - 1.0, 0.0, W - 1.0])
    ys = np.array([0.0, 0.0, H - 1.0, H - 1.0])
    u = h[..., 0, 0, None] * xs + h[..., 0, 1, None] * ys + h[..., 0, 2, None]
    v = h[..., 1, 0, None] * xs + h[..., 1, 1, None] * ys + h[..., 1, 2, None]
    w = h[..., 2, 0, None] * xs + h[..., 2, 1, None] * ys + h[..., 2, 2, None]
    same = (np.all(w > 0, axis=-1) | np.all(w < 0, axis=-1))
    with np.errstate(divide="ignore", invalid="ignore"):
        px = u / w * W / max(H - 1, 1) - 0.5
        py = v / w * H / max(W - 1, 1) - 0.5
    x0 = np.clip(np.floor(px.min(-1)), 0, W - 1)
    x1 = np.clip(np.floor(px.max(-1)) + 1, 0, W - 1)
    y0 = np.clip(np.floor(py.min(-1)), 0, H - 1)
    y1 = np.clip(np.floor(py.max(-1)) + 1, 0, H - 1)
    off = (px.max(-1) < -1) | (px.min(-1) > W) | (py.max(-1) < -1) | (py.min(-1) > H)
    box = np.stack([x0, x1, y0, y1], -1)
    box[~same] = [0, W - 1, 0, H - 1]
    box[same & off] = [0, -1, 0, -1]  # every tap outside the image: nothing read
    return box.astype(np.int64)


def needed_bytes(homs: np.ndarray, H: int, W: int, union: bool = False) -> int:
    """HBM bytes of texels the render actually samples (sampled_boxes x 16 B) + the frames
    written (12 B per pixel per view).  union: views sharing one MPI read it once, so each
    plane counts the bounding box of its views' boxes (an upper bound of their union)."""
    box = sampled_boxes(homs, H, W)
    V = box.shape[0]
    if union:
        box = np.stack([box[..., 0].min(0), box[..., 1].max(0), box[..., 2].min(0), box[..., 3].max(0)], -1)[None]
    area = np.clip(box[..., 1] - box[..., 0] + 1, 0, None) * np.clip(box[..., 3] - box[..., 2] + 1, 0, None)
    return int(area.sum()) * 16 + V * H * W * 12


# ---------------------------------------------------------------------------
# CPU baseline
# ---------------------------------------------------------------------------

def host_cores():
    """(threads to use, description): the cores this process may run on (affinity, cgroup
    CPU quota) -- the box's CPU share -- capped by OMP_NUM_THREADS when the box sets it."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(usable, omp) if omp > 0 else usable
    return threads, {"host_nproc": nproc, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                     "omp_num_threads_env": omp or None, "threads_used": threads}


def cpu_baseline(view_dev: torch.Tensor, homs_all: torch.Tensor, budget_s: float, check_frames):
    """The oracle's C restatement (bit-exact to the reference) on this host's cores, on a
    bounded sample: whole views of the same MPI, as many as fit ~budget_s."""
    from oracle import oracle
    threads, cores = host_cores()
    mpi = view_dev.cpu().numpy()[None]          # [1,H,W,P,4]
    H, W = mpi.shape[1], mpi.shape[2]
    views, t_total, outs = 0, 0.0, []
    while views == 0 or (t_total < budget_s and views < homs_all.shape[0]):
        h = homs_all[views:views + 1].numpy()
        t0 = time.perf_counter()
        o = oracle.render(mpi, h, threads)
        t_total += time.perf_counter() - t0
        outs.append(o)
        views += 1
    mism = sum(1 for i, o in enumerate(outs[:len(check_frames)]) if not np.array_equal(o, check_frames[i]))
    return {"value": views * H * W / 1e6 / t_total, "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{views} full view(s) of the config-4 1024x1024x128 MPI (camera-path poses 0..{views - 1}) "
                      f"with the oracle's C restatement (oracle/mpiv_oracle.c, {threads} OpenMP threads), "
                      f"{t_total:.1f} s",
            "host": cores, "gpu_frames_bit_exact_vs_cpu": mism == 0,
            "reference_cpu": {"value": REF_CPU["c4_Mpix_s"], "unit": "Mpix/s", "cores": REF_CPU["cores"],
                              "s_per_view": REF_CPU["c4_s_per_view"], "source": REF_CPU["source"]}}


# ---------------------------------------------------------------------------
# legs
# ---------------------------------------------------------------------------

def single_view_leg(packed, H, W, P, h_sv, dev, stream):
    """One view per launch (every texel crosses HBM once): the north-star HBM bar."""
    one = torch.empty((1, H, W, 3), device=dev)
    launch = lambda: _lib._call("mpiv_render_packed", packed, H, W, P, h_sv, 1, one, _lib._stream(dev))  # noqa: E731
    warm(launch, stream)
    mark("sv", dev)
    ms = event_ms(launch, 20, stream)
    mark("untimed", dev)
    alg = P * H * W * 16 + H * W * 12
    gbs, frac = hbm(alg, ms)
    kname, grid = _lib.route("render_packed", H, W, P, 1)
    res = {"workload": "config 4 MPI, one view per launch", "kernel_ms": round(ms, 4), "alg_bytes": alg,
           "alg_def": "P*H*W*16 + H*W*12", "achieved_gbs": gbs, "peak": HBM_PEAK_GBS, "frac": frac, "bound": "hbm"}
    res.update(prof_fields(kname, grid, alg, ms, "sv"))
    return res


def config2_leg(dev, stream, n=20):
    """BASELINE config 2: a 32-plane 1024x576 MPI broadcast to 64 target views, one launch
    of all 64 from the packed MPI (the drop-in packs a stride-0 batch once)."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    V = len(c["poses"])
    packed = _lib.pack_planes(gen_view(H, W, P, c["seed"], dev))
    homs = _host.render_homographies(configs.f32(c["poses"]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]] * V), V).to(dev)
    out = torch.empty((V, H, W, 3), device=dev)
    launch = lambda: _lib._call("mpiv_render_packed", packed, H, W, P, homs, V, out, _lib._stream(dev))  # noqa: E731
    warm(launch, stream)
    mark("c2", dev)
    ms = event_ms(launch, n, stream)
    mark("untimed", dev)
    alg = V * (P * H * W * 16 + H * W * 12)
    gbs, frac = hbm(alg, ms)
    kname, grid = _lib.route("render_packed", H, W, P, V)
    hn = homs.cpu().numpy()
    need_views = needed_bytes(hn, H, W)
    need_union = needed_bytes(hn, H, W, union=True)
    res = {"workload": "BASELINE config 2: 32-plane 1024x576 MPI, 64 target views in one launch",
           "kernel_ms": round(ms, 4), "Mpix_per_s": round(V * H * W / 1e6 / (ms * 1e-3), 1),
           "baseline_bar_Mpix_s": 9160, "alg_bytes": alg, "alg_def": "V*(P*H*W*16 + H*W*12) (SURVEY §8d)",
           "alg_gbs": gbs, "alg_frac": frac,
           "alg_frac_note": "the 64 views share one MPI through L2, so the per-view formula can exceed 1 of HBM",
           # the reference's swapped normalisation (utils.py:186-188) maps output row y to MPI row
           # ~y*H/(W-1): a 576x1024 view samples only ~56 % of the MPI's rows
           "needed_bytes_per_view_sum": need_views, "needed_frac_per_view_sum": hbm(need_views, ms)[1],
           "needed_bytes_union": need_union, "needed_union_frac": hbm(need_union, ms)[1],
           "needed_def": "texel boxes each (view, plane) samples (homographies at the frame corners; the map is "
                         "linear-fractional) x 16 B + frames; union: one read of the views' bounding box per plane"}
    res.update(prof_fields(kname, grid, alg, ms, "c2"))
    del packed, out
    return res


def config3_leg(dev, stream, n=20):
    """BASELINE config 3: plane-sweep volume of 5 source 1024x768 images into 64 planes through
    the drop-in plane_sweep_torch (host Ki/proj + one mpiv_plane_sweep launch), and that
    launch alone."""
    import mpi_vision_amd as mv
    c = configs.config3()
    S, H, W, D = c["S"], c["H"], c["W"], c["D"]
    g = torch.Generator(device=dev).manual_seed(c["seed"])
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S).to(dev)
    pose = configs.f32(c["poses"]).to(dev)
    depths = list(c["depths"])
    vol = mv.plane_sweep_torch(img, depths, pose, K)
    warm(lambda: mv.plane_sweep_torch(img, depths, pose, K), stream)
    mark("c3_dropin", dev)
    dropin_ms = span_ms(lambda: mv.plane_sweep_torch(img, depths, pose, K), n, stream)
    mark("untimed", dev)
    ki, proj = _host.psv_matrices(K.cpu(), K.cpu(), pose.cpu())
    ki, proj = ki.to(dev), proj.to(dev)
    dd = configs.f32(depths).to(dev)
    out = torch.empty((S, H, W, D * 3), device=dev)
    launch = lambda: _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, dd, D, H, W,  # noqa: E731
                                out, _lib._stream(dev))
    launch()
    same = bool(torch.equal(out.view(torch.int32), vol.view(torch.int32)))
    # every timed launch counts: the warm-up (WARM_MS of untimed launches), then the mean of 3n
    # back-to-back launches -- the rate this write-heavy kernel sustains (the mean of
    # every timed launch, not a best case; the thirds show any drift)
    nwarm = warm(launch, stream)
    mark("c3", dev)
    ms_each = event_ms(launch, 3 * n, stream, each=True)
    mark("untimed", dev)
    ms = float(np.mean(ms_each))
    alg = S * H * W * 12 + S * D * H * W * 12
    gbs, frac = hbm(alg, ms)
    kname, grid = _lib.route("plane_sweep", S, H, W, 3, D, H, W)
    # four of the sources into the notebook dataset's 10 planes (ipynb cell 8 L73-75: inv_depths(1, 100,
    # 10)); four, not five, so that its launches have their own grid size in the rocprof summary
    D10, S10 = 10, 4
    d10 = configs.f32(configs.inv_depths(1, 100, D10)).to(dev)
    out10 = torch.empty((S10, H, W, D10 * 3), device=dev)
    img10 = img[:S10]
    launch10 = lambda: _lib._call("mpiv_plane_sweep", img10, _lib._strides(img10), S10, H, W, 3, ki, proj, d10,  # noqa: E731
                                  D10, H, W, out10, _lib._stream(dev))
    warm(launch10, stream)
    mark("c3_ten", dev)
    ms10 = event_ms(launch10, n, stream)
    mark("untimed", dev)
    alg10 = S10 * H * W * 12 + S10 * D10 * H * W * 12
    k10, g10 = _lib.route("plane_sweep", S10, H, W, 3, D10, H, W)
    ten = {"workload": "4 of config 3's sources into 10 depth planes (the notebook dataset's depth count)",
           "kernel_ms": round(ms10, 4), "alg_bytes": alg10, "achieved_gbs": hbm(alg10, ms10)[0],
           "frac": hbm(alg10, ms10)[1], "bound": "hbm"}
    ten.update(prof_fields(k10, g10, alg10, ms10, "c3_ten"))
    del out10
    res = {"workload": "BASELINE config 3: PSV of 5 source 1024x768x3 images into 64 depth planes "
                       "(plane_sweep_torch, utils.py:452-471)",
           "kernel_ms": round(ms, 4), "kernel_ms_def": f"mean of {3 * n} back-to-back launches after {nwarm} untimed ({WARM_MS:.0f} ms)",
           "kernel_ms_first_last_third": [round(float(np.mean(ms_each[:n])), 4), round(float(np.mean(ms_each[-n:])), 4)],
           "dropin_ms": round(dropin_ms, 4),
           "Mplanepix_per_s": round(S * D * H * W / 1e6 / (ms * 1e-3), 1),
           "alg_bytes": alg, "alg_def": "S*Hs*Ws*C*4 + S*D*Ht*Wt*C*4 (SURVEY §8d)", "achieved_gbs": gbs,
           "peak": HBM_PEAK_GBS, "frac": frac, "bound": "hbm", "baseline_bar_ms": 0.64,
           "dropin_equals_kernel": same,
           "reference_cpu": {"s": REF_CPU["c3_s"], "cores": REF_CPU["cores"], "source": REF_CPU["source"]}}
    res.update(prof_fields(kname, grid, alg, ms, "c3"))
    res["ten_planes"] = ten
    del img, out, vol
    return res


def notebook_leg(dev, stream, n=50):
    """The reference's only real caller at its own size (fast-torch-stereo-vision.ipynb
    cell 8 L89-90: img_size 224, num_planes 10, bs 1): the dataset's PSV
    (plane_sweep_torch_one at inv_depths(1, 100, 10), cell 8 L73-75), the loss's render
    (mpi_render_view_torch, cell 12 L42) and the render's training step (forward with
    autograd + backward), all through the drop-in functions."""
    import mpi_vision_amd as mv
    S = N = 224
    P = 10
    depths = mv.inv_depths(1, 100, P)
    f = configs.focal_from_fov(N)
    K = configs.f32(configs.intrinsics_matrix(f, f, N / 2.0, N / 2.0)).to(dev)
    pose = configs.f32(configs.pose_from(configs.rot_y(1.0), (0.05, -0.02, 0.03))).to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    img = torch.rand((S, N, 3), generator=g, device=dev)
    psv = lambda: mv.plane_sweep_torch_one(img, depths, pose, K)  # noqa: E731
    warm(psv, stream)
    psv_ms = span_ms(psv, n, stream)
    ki, proj = _host.psv_matrices(K.cpu()[None], K.cpu()[None], pose.cpu()[None])
    ki, proj = ki.to(dev), proj.to(dev)
    dd = configs.f32(depths).to(dev)
    out = torch.empty((1, S, N, P * 3), device=dev)
    img4 = img[None]
    launch = lambda: _lib._call("mpiv_plane_sweep", img4, _lib._strides(img4), 1, S, N, 3, ki, proj, dd, P, S, N,  # noqa: E731
                                out, _lib._stream(dev))
    warm(launch, stream)
    mark("nb", dev)
    psv_kernel_ms = event_ms(launch, n, stream)
    mark("untimed", dev)
    psv_alg = S * N * 12 + P * S * N * 12
    mpi = configs.synthetic_mpi(1, S, N, P, 9).to(dev)
    planes = configs.f32(depths).to(dev)
    poses = pose[None]
    Kb = K[None]
    rend = lambda: mv.mpi_render_view_torch(mpi, poses, planes, Kb)  # noqa: E731
    warm(rend, stream)
    render_ms = span_ms(rend, n, stream)
    leaf = mpi.clone().requires_grad_(True)
    dout = torch.rand((1, S, N, 3), generator=g, device=dev)

    def train_step():
        o = mv.mpi_render_view_torch(leaf, poses, planes, Kb)
        o.backward(dout)
        leaf.grad = None
    warm(train_step, stream)
    # host-bound (PyTorch's autograd engine around two small launches): five spans of n back-to-back
    # steps, the median reported (one span can catch a garbage-collector pause; all five are listed)
    train_reps = [span_ms(train_step, n, stream) for _ in range(5)]
    train_ms = float(np.median(train_reps))
    # the same step captured in HIP graphs (torch.cuda.make_graphed_callables): the forward and the
    # backward each replay as one graph, so no per-step Python / autograd host work remains
    graphed = {}
    try:
        class _RenderStep(torch.nn.Module):
            def forward(self, m):
                return mv.mpi_render_view_torch(m, poses, planes, Kb)
        leaf.grad = None
        mv.mpi_render_view_torch(leaf, poses, planes, Kb).backward(dout)
        eager_grad = leaf.grad.clone()
        leaf.grad = None
        # the leaf's AccumulateGrad node dates from the eager steps on the bench stream; the capture's
        # warm-up runs on a side stream, which PyTorch reports as a stream mismatch (expected here)
        if hasattr(torch.autograd.graph, "set_warn_on_accumulate_grad_stream_mismatch"):
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        gfn = torch.cuda.make_graphed_callables(_RenderStep(), (leaf,))

        def gstep():
            gfn(leaf).backward(dout)
            leaf.grad = None
        gfn(leaf).backward(dout)
        torch.cuda.synchronize()
        same = bool(torch.equal(leaf.grad.view(torch.int32), eager_grad.view(torch.int32)))
        leaf.grad = None
        warm(gstep, stream)
        g_reps = [span_ms(gstep, n, stream) for _ in range(5)]
        graphed = {"train_step_graphed_ms": round(float(np.median(g_reps)), 4),
                   "train_step_graphed_ms_reps": [round(x, 4) for x in g_reps], "graphed_grad_bit_identical": same,
                   "graphed_def": "the same step through torch.cuda.make_graphed_callables (HIP graphs: forward and "
                                  "backward replayed as one graph each)"}
    except RuntimeError as e:
        graphed = {"train_step_graphed_error": f"{type(e).__name__}: {e}"[:300]}
    kname, grid = _lib.route("plane_sweep", 1, S, N, 3, P, S, N)
    r_alg = P * S * N * 16 + S * N * 12
    res = {"workload": "notebook shape (ipynb cell 8 L89-90): 224x224, 10 planes, bs 1",
           "psv_dropin_ms": round(psv_ms, 4), "psv_kernel_ms": round(psv_kernel_ms, 4),
           "psv_alg_bytes": psv_alg, "psv_frac": hbm(psv_alg, psv_kernel_ms)[1],
           "render_dropin_ms": round(render_ms, 4), "render_alg_bytes": r_alg,
           "train_step_ms": round(train_ms, 4), "train_step_ms_reps": [round(x, 4) for x in train_reps],
           "train_step_def": "mpi_render_view_torch forward (autograd, checkpoints) + backward through the drop-in; "
                             f"median of 5 spans of {n} back-to-back steps",
           "note": "8 MB of texels: launch-latency-bound at this size", "psv": prof_fields(kname, grid, psv_alg,
                                                                                             psv_kernel_ms, "nb")}
    res.update(graphed)
    del mpi, leaf, out
    return res


def guarded(fn, *args):
    """An auxiliary leg: a Python-level failure (an entry point's error, a shape bug) is recorded
    in the line instead of ending the run before the headline is printed."""
    try:
        return fn(*args)
    except (RuntimeError, ValueError, AssertionError, TypeError) as e:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        return {"error": f"{type(e).__name__}: {e}"[:400]}


def u8_leg(dev, stream, V, homs_sv, homs_v, n=10):
    """The 8-bit texel path (the reference's own test MPI is 8-bit, test/rgba_*.png,
    read as u8/255, utils.py:324-331): a config-4-shape u8 MPI (counter-based synthetic bytes,
    synth.hip, packed at 4 B per texel) rendered one view per launch (the HBM-bound case) and
    V views per launch (the headline's camera-path views).  Self-check: the single-view frame
    equals the float render of the same MPI as u8/255 (IEEE division on the host) bit for bit."""
    c4 = configs.config4()
    H, W, P = c4["H"], c4["W"], c4["P"]
    pk = _lib.synth_mpi_packed_u8(c4["seed"], H, W, 0, P, dev)
    one = torch.empty((1, H, W, 3), device=dev)
    many = torch.empty((V, H, W, 3), device=dev)
    l1 = lambda: _lib._call("mpiv_render_packed_u8", pk, H, W, P, homs_sv, 1, one, _lib._stream(dev))  # noqa: E731
    lv_u8 = lambda: _lib._call("mpiv_render_packed_u8", pk, H, W, P, homs_v, V, many, _lib._stream(dev))  # noqa: E731
    warm(l1, stream)
    mark("u8_sv", dev)
    ms1 = event_ms(l1, 20, stream)
    mark("untimed", dev)
    # V views per launch: the route render_packed_u8 takes there (>= U8_FLOAT_MIN_VIEWS): the float
    # kernel on the MPI's exact float copy, converted once per MPI (timed separately, outside)
    route_float = V >= _lib.U8_FLOAT_MIN_VIEWS
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    fcopy = _lib.u8_float_copy(pk) if route_float else None
    ev1.record(stream)
    torch.cuda.synchronize()
    convert_ms = ev0.elapsed_time(ev1) if route_float else None
    lv = (lambda: _lib._call("mpiv_render_packed", fcopy, H, W, P, homs_v, V, many, _lib._stream(dev))) \
        if route_float else lv_u8  # noqa: E731
    warm(lv, stream)
    mark("u8_mv", dev)
    msv = event_ms(lv, n, stream)
    mark("untimed", dev)
    want = many.clone()
    warm(lv_u8, stream)
    mark("u8_kernel", dev)
    msv_u8 = event_ms(lv_u8, n, stream)
    mark("untimed", dev)
    same_v = bool(torch.equal(want.view(torch.int32), many.view(torch.int32)))
    del fcopy, want
    _lib.clear_u8_float_copies()
    # float packed copy of u8/255 (numpy fp32 division is IEEE) for the bit-exact self-check
    f = (pk.view(torch.uint8).cpu().numpy().reshape(P, H + 4, W + 4, 4).astype(np.float32) / np.float32(255.0))
    fpk = torch.from_numpy(f).to(dev)
    del f
    ref = torch.empty((1, H, W, 3), device=dev)
    _lib._call("mpiv_render_packed", fpk, H, W, P, homs_sv, 1, ref, _lib._stream(dev))
    same = bool(torch.equal(ref.view(torch.int32), one.view(torch.int32)))
    del fpk, ref
    alg1 = P * H * W * 4 + H * W * 12
    k1, g1 = _lib.route("render_packed_u8", H, W, P, 1)
    kv, gv = _lib.route("render_packed" if route_float else "render_packed_u8", H, W, P, V)
    ku, gu = _lib.route("render_packed_u8", H, W, P, V)
    sv = {"kernel_ms": round(ms1, 4), "alg_bytes": alg1, "alg_def": "P*H*W*4 (u8 texels) + H*W*12",
          "achieved_gbs": hbm(alg1, ms1)[0], "frac": hbm(alg1, ms1)[1], "bound": "hbm",
          "frame_equals_float_render_of_u8_over_255": same}
    sv.update(prof_fields(k1, g1, alg1, ms1, "u8_sv"))
    algv = V * alg1
    mv_ = {"views": V, "kernel_ms": round(msv, 4), "Mpix_per_s": round(V * H * W / 1e6 / (msv * 1e-3), 1),
           "route": ("float kernel on the MPI's exact float copy (render_packed_u8 at >= "
                     f"{_lib.U8_FLOAT_MIN_VIEWS} views per launch)") if route_float else "u8 kernel",
           "u8_to_float_copy_ms_once": round(convert_ms, 4) if convert_ms is not None else None,
           "frames_equal_u8_kernel": same_v,
           "alg_bytes": algv, "alg_gbs": hbm(algv, msv)[0],
           "alg_frac_note": "the views share one MPI through L2: the per-view formula can exceed 1 of HBM"}
    mv_.update(prof_fields(kv, gv, algv, msv, "u8_mv"))
    mv_["u8_kernel"] = {"kernel_ms": round(msv_u8, 4)}
    mv_["u8_kernel"].update(prof_fields(ku, gu, algv, msv_u8, "u8_kernel"))
    del pk, one, many
    torch.cuda.empty_cache()
    return {"workload": "config-4-shape 8-bit MPI (1024x1024x128, 4-B texels): one view and the camera-path "
                        f"launch of {V} views", "single_view": sv, "multi_view": mv_}


def netout_needed_bytes(homs: np.ndarray, H: int, W: int) -> int:
    """Bytes the fused net-output render of one view needs: each plane's w / a channels over its
    sampled texel box (sampled_boxes) x 8 B, bg / reference image over the planes' bounding box x 24 B,
    the frame written."""
    box = sampled_boxes(homs, H, W)[0]
    area = np.clip(box[:, 1] - box[:, 0] + 1, 0, None) * np.clip(box[:, 3] - box[:, 2] + 1, 0, None)
    live = area > 0
    if live.any():
        ub = (int(box[live, 0].min()), int(box[live, 1].max()), int(box[live, 2].min()), int(box[live, 3].max()))
    else:
        ub = (0, -1, 0, -1)
    return int(area.sum()) * 8 + max(ub[1] - ub[0] + 1, 0) * max(ub[3] - ub[2] + 1, 0) * 24 + H * W * 12


def netout_leg(dev, stream, n=20):
    """The network output rendered in one kernel (notebook mpi_from_net_output, ipynb cell 10
    L79-111, fused into mpi_render_view_torch: render_netout_kernel) at config 2's size
    (1024x576, 32 planes), one view; self-check against the two-step drop-ins
    (assemble_mpi + render), bit for bit."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(c["seed"])
    pred = torch.rand((1, 2 * P + 3, H, W), generator=g, device=dev) * 2 - 1
    fg = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    homs = _host.render_homographies(configs.f32(c["poses"][5:6]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1).to(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    launch = lambda: _lib._call("mpiv_render_net_output", pred, _lib._strides(pred), fg, _lib._strides(fg), 1,  # noqa: E731
                                H, W, P, homs, out, _lib._stream(dev))
    warm(launch, stream)
    mark("netout", dev)
    ms = event_ms(launch, n, stream)
    mark("untimed", dev)
    two = _lib.render(_lib.assemble_mpi(pred, fg, P), homs)
    same = bool(torch.equal(two.view(torch.int32), out.view(torch.int32)))
    alg = H * W * ((2 * P + 3) * 4 + 12 + 12)
    kname, grid = _lib.route("render_net_output", 1, H, W, P)
    res = {"workload": "network output [1, 2P+3, 576, 1024] (P = 32) + reference image -> rendered view, one kernel",
           "kernel_ms": round(ms, 4), "alg_bytes": alg, "alg_def": "H*W*((2P+3)*4 + 12 + 12): prediction + "
           "reference image read, frame written", "achieved_gbs": hbm(alg, ms)[0], "frac": hbm(alg, ms)[1],
           "bound": "hbm", "equals_assemble_then_render": same}
    # the bytes the reference's mapping samples (VERDICT r5 #5's measure, as for configs 2 and 5): each
    # plane's w / a over its sampled box (8 B per texel), bg / ref image over the planes' bounding box
    # (24 B per texel), the frame written
    need = netout_needed_bytes(homs.cpu().numpy(), H, W)
    res.update({"needed_bytes": need, "needed_frac": hbm(need, ms)[1],
                "needed_def": "w / a over each plane's sampled texel box (bench.sampled_boxes) x 8 B + bg / ref image "
                              "over the planes' bounding box x 24 B + the frame written"})
    res.update(prof_fields(kname, grid, alg, ms, "netout"))
    del out, two
    res["training"] = netout_training(dev, stream, pred, fg, c)
    del pred, fg
    return res


def netout_training(dev, stream, pred0, fg0, c, n=20):
    """The notebook losses' training step (ipynb cell 12 L7-11 / L38-42: mpi_from_net_output ->
    mpi_render_view_torch -> backward) at config 2's size, through the drop-ins under autograd:
    fused (mpi_render_net_output_torch: render_netout_kernel + checkpoints; the backward re-assembles
    the MPI) against the two-step chain (assemble, training render, backward, assembly backward).
    Same gradients bit for bit (checked); HBM bytes per step and the memory the autograd graph holds
    between forward and backward (saved tensors + frame) beside the times."""
    import mpi_vision_amd as mv
    H, W, P = c["H"], c["W"], c["P"]
    pose = configs.f32(c["poses"][5:6]).to(dev)
    K = configs.f32([c["K"]]).to(dev)
    planes = configs.f32(c["depths"]).to(dev)
    dout = torch.rand((1, H, W, 3), generator=torch.Generator(device=dev).manual_seed(3), device=dev) * 2 - 1
    pred = pred0.clone().requires_grad_(True)
    fg = fg0.clone().requires_grad_(True)
    dep = {"mpi_planes": torch.zeros((1, P), device=dev), "ref_img": fg}

    def fused_fwd():
        return mv.mpi_render_net_output_torch(pred, fg, pose, planes, K)

    def two_fwd():
        return mv.mpi_render_view_torch(mv.mpi_from_net_output(pred, dep), pose, planes, K)

    def step(fwd):
        pred.grad = fg.grad = None
        fwd().backward(dout)

    res = {"workload": "config-2-size training step (1024x576, 32 planes, 1 view): forward + backward through the "
                       "drop-ins, d network output and d reference image"}
    grads = {}
    for name, fwd in (("fused", fused_fwd), ("two_step", two_fwd)):
        step(fwd)
        torch.cuda.synchronize()
        grads[name] = (pred.grad.clone(), fg.grad.clone())
        pred.grad = fg.grad = None
        torch.cuda.synchronize()
        m0 = torch.cuda.memory_allocated(dev)
        o = fwd()
        torch.cuda.synchronize()
        held = torch.cuda.memory_allocated(dev) - m0
        del o
        warm(lambda: step(fwd), stream)
        mark("nt_" + name, dev)
        ms = span_ms(lambda: step(fwd), n, stream)
        mark("untimed", dev)
        res[name] = {"step_ms": round(ms, 4), "graph_bytes_between_fwd_and_bwd": int(held),
                     "rocprof_kernels": prof_tag_kernels("nt_" + name, n)}
    res["grads_bit_identical"] = bool(torch.equal(grads["fused"][0].view(torch.int32), grads["two_step"][0].view(torch.int32))
                                      and torch.equal(grads["fused"][1].view(torch.int32),
                                                      grads["two_step"][1].view(torch.int32)))
    mpi = P * H * W * 16
    net = H * W * (2 * P + 3) * 4 + H * W * 12   # prediction + reference image
    ck = (P + 7) // 8 * H * W * 16
    frame = H * W * 12
    # algorithmic HBM bytes per step, kernel by kernel (render backward counted as MPI read + d MPI
    # written + d frame read, its workspace traffic excluded, as in the training leg)
    bwd = 2 * mpi + frame
    asm_bwd = mpi + net + net
    two = (net + mpi) + (mpi + ck + frame) + bwd + asm_bwd
    fused = (net + ck + frame) + (net + mpi) + bwd + asm_bwd
    res.update({"alg_bytes_two_step": two, "alg_bytes_fused": fused,
                "alg_bytes_def": "assemble (pred+ref read, MPI written) + training render (MPI read, checkpoints + "
                                 "frame written) + render backward (MPI read, d MPI written, d frame read) + assembly "
                                 "backward (d MPI, pred + ref read, d pred + d ref written); fused: render_netout with "
                                 "checkpoints instead of assemble + training render, the assembly moved into the "
                                 "backward"})
    if res["fused"]["step_ms"] and res["two_step"]["step_ms"]:
        res["fused_over_two_step_time"] = round(res["fused"]["step_ms"] / res["two_step"]["step_ms"], 3)
    del pred, fg, grads
    torch.cuda.empty_cache()
    return res


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
    # kernel figures: the entry points on preallocated outputs, launched back to back (the
    # drop-ins' per-call host work -- checks, allocation, ~30-50 us -- would otherwise show up as
    # device idle time between each pair of events); the drop-in call is reported beside them
    f_out = torch.empty((1, H, W, 3), device=dev)
    f_ck = torch.empty_like(ck)
    st = _lib._strides(mpi)
    fwd = lambda: _lib._call("mpiv_render_train", mpi, st, 1, H, W, P, homs, f_out, f_ck,  # noqa: E731
                             _lib._stream(dev))
    inf = lambda: _lib._call("mpiv_render", mpi, st, 1, H, W, P, homs, f_out, _lib._stream(dev))  # noqa: E731
    warm(fwd, stream)
    mark("train_fwd", dev)
    fwd_ms = span_ms(fwd, n, stream)
    mark("untimed", dev)
    warm(inf, stream)
    mark("train_inf", dev)
    inf_ms = span_ms(inf, n, stream)
    mark("untimed", dev)
    warm(lambda: _lib.render(mpi, homs), stream)
    mark("train_inf_dropin", dev)
    inf_dropin_ms = event_ms(lambda: _lib.render(mpi, homs), n, stream)
    mark("untimed", dev)
    same_ck = bool(torch.equal(f_ck.view(torch.int32), ck.view(torch.int32)))
    del f_ck
    g1 = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
    warm(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck), stream)
    mark("train_bwd", dev)
    bwd_ms = span_ms(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck), n, stream)
    mark("untimed", dev)
    g2 = _lib.render_backward(mpi, homs, dout, workspace=ws)
    warm(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws), stream)
    mark("train_bwd_nockpt", dev)
    bwd2_ms = span_ms(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws), n, stream)
    mark("untimed", dev)
    # the smallest workspace (plane groups, round 4): same gradient, d samples of one group resident
    ws_min = torch.empty(_lib.load().mpiv_render_backward_workspace_size_min(H, W, P), dtype=torch.uint8, device=dev)
    g3 = _lib.render_backward(mpi, homs, dout, workspace=ws_min, ckpt=ck)
    warm(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws_min, ckpt=ck), stream)
    mark("train_bwd_minws", dev)
    bwd3_ms = span_ms(lambda: _lib.render_backward(mpi, homs, dout, workspace=ws_min, ckpt=ck), n,
                      stream)
    mark("untimed", dev)
    same_min = bool(torch.equal(g1.view(torch.int32), g3.view(torch.int32)))
    ws_min_gb = round(ws_min.numel() / 1e9, 3)
    del g3, ws_min
    flag = int(ws[_lib.bwd_flag_offset(H, W, P):][:4].view(torch.int32).item())
    aborted = _lib.render_backward_status(ws, H, W, P)
    same = bool(torch.equal(g1.view(torch.int32), g2.view(torch.int32)))
    mpi_bytes = P * H * W * 16
    f_alg = mpi_bytes + H * W * 12
    b_alg = 2 * mpi_bytes + H * W * 12
    kname, grid = _lib.route("render", 1, H, W, P)
    res = {"workload": "BASELINE config 4 MPI (1024x1024x128), one non-broadcast view: training forward + backward",
           "inference_ms": round(inf_ms, 4), "inference_frac": hbm(f_alg, inf_ms)[1],
           "inference_dropin_ms": round(inf_dropin_ms, 4),
           "timing": "forward / inference: entry points on preallocated outputs; all: n calls back to back, "
                     "device span / n",
           "forward_ckpt_bit_identical": same_ck,
           "forward_ms": round(fwd_ms, 4), "backward_ms": round(bwd_ms, 4),
           "backward_no_ckpt_ms": round(bwd2_ms, 4), "step_ms": round(fwd_ms + bwd_ms, 4),
           "forward_alg_bytes": f_alg, "forward_hbm_frac": hbm(f_alg, fwd_ms)[1],
           "backward_alg_bytes": b_alg,
           "backward_alg_def": "MPI read + d MPI written + d frame read (workspace traffic not counted)",
           "backward_hbm_frac": hbm(b_alg, bwd_ms)[1],
           "workspace_GB": round(ws.numel() / 1e9, 3), "fallback_flag": flag, "fallback_aborted_views": aborted,
           "backward_min_workspace_ms": round(bwd3_ms, 4), "workspace_min_GB": ws_min_gb,
           "min_workspace_grad_bit_identical": same_min,
           "min_workspace_def": "mpiv_render_backward_workspace_size_min: plane groups of 32, one group's d samples resident",
           "ckpt_grad_bit_identical": same, "inference": prof_fields(kname, grid, f_alg, inf_ms, "train_inf"),
           # per-kernel rocprof attribution of each timed sub-leg (phase-tagged dispatches,
           # tools/parse_prof.py): chain, gather, ... with dispatches and ms per call
           "rocprof_kernels": {t: prof_tag_kernels(t, n) for t in
                               ("train_fwd", "train_bwd", "train_bwd_nockpt", "train_bwd_minws")}}
    fk = prof_for(_lib.route("render_train", 1, H, W, P)[0], _lib.route("render_train", 1, H, W, P)[1], "train_fwd")
    if fk:
        res["forward_rocprof_ms"] = round(fk["avg_ns"] / 1e6, 4)
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
        kname, grid = _lib.route("render_packed", H, W, P, 1)
    else:
        ct = torch.empty((1, H, W, 4), device=dev)
        launch = lambda: _lib._call("mpiv_render_packed_ct", packed, H, W, p1 - p0, 0, p1 - p0,  # noqa: E731
                                    int(rank == 0), hl, 1, ct, _lib._stream(dev))
        xstats = {}
        # the band pipeline by default (MPIV_PLANE_PIPELINE=0: the one-shot all-to-all path)
        pipe = os.environ.get("MPIV_PLANE_PIPELINE", "1") != "0"
        step = lambda: parallel.render_plane_sharded(packed, hl, H, stats=xstats, pipelined=pipe)  # noqa: E731
        shard_bytes = (p1 - p0) * H * W * 16 + H * W * 16
        kname, grid = _lib.route("render_packed_ct", H, W, p1 - p0, 1)
    warm(launch, stream)
    mark("c5_kernel", dev)
    kern_ms = event_ms(launch, 3, stream)
    mark("untimed", dev)
    if world > 1 and fault_injected("c5_hang", rank):
        time.sleep(1e6)  # the peers block in the band exchange
    if world > 1 and fault_injected("c5_raise", rank):
        raise RuntimeError("MPIV_BENCH_FAULT=c5_raise: injected exchange failure")
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
    kern_all = all_ranks(kern_ms, world, dev)
    hn = homs[:, p0:p1].numpy()
    shard_need = needed_bytes(hn, H, W) if world == 1 else needed_bytes(hn, H, W) + H * W * 4
    res = {"workload": "BASELINE config 5: 256-plane 4096x2160 MPI (36.2 GB), 1 pose, plane-sharded",
           "value": round(steps * H * W / 1e6 / elapsed, 2), "unit": "Mpix/s", "n_gpus": world,
           "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "scaling": "strong",
           "data": "synthetic (counter-based per-shard generator, synth.hip, seed 0)",
           "planes_per_gpu": p1 - p0, "shard_kernel_ms": round(max(kern_all), 3),
           "per_rank_shard_kernel_ms": [round(x, 3) for x in kern_all],
           "shard_alg_bytes": shard_bytes,
           "shard_hbm_frac": hbm(shard_bytes, max(kern_all))[1],
           # the bytes the reference's mapping actually samples (utils.py:186-188: output row y reads
           # MPI row ~y*H/(W-1), so a 4096x2160 frame touches only MPI rows ~0..1200 of each plane)
           "shard_needed_bytes": shard_need, "shard_needed_frac": hbm(shard_need, max(kern_all))[1],
           "needed_def": "texel boxes each plane samples (homographies at the frame corners; the map is "
                         "linear-fractional) x 16 B + the frame / partial written",
           "parallelism": "single GPU, sequential render" if world == 1 else
           f"plane-sharded x{world}: (C,T) partials + band all-to-all + ordered combine + gather",
           "frame_sha16": sha16(frame) if rank == 0 else None}
    if world > 1:
        # the band exchange is pipelined with the render (parallel.render_plane_sharded_pipelined):
        # what the exchange adds over the slowest rank's render is the exposed part
        step_ms = elapsed / steps * 1e3
        sent = max(all_ranks(float(xstats.get("bytes_sent", 0)), world, dev))
        res.update({"exchange": "pipelined: G-1 batched pair exchanges of row bands, each posted as soon as its "
                                "band is rendered (mpiv_render_packed_ct_rows)",
                    "bytes_sent_per_rank": int(sent), "exchange_exposed_ms": round(step_ms - max(kern_all), 3),
                    "exchange_gbs_over_step": round(sent / (step_ms * 1e-3) / 1e9, 2)})
    res.update(prof_fields(kname, grid, shard_bytes, max(kern_all), "c5_kernel"))
    if res.get("traffic"):
        res["traffic_over_needed"] = round(res["traffic"] / shard_need, 3)
    del packed
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))  # before any GPU call in this process
    world, rank, dev, backend = dist_setup(args)
    torch.cuda.set_device(dev)
    legs = args.legs
    c4 = configs.config4()
    H, W, P = c4["H"], c4["W"], c4["P"]
    V = args.views
    n_path = len(c4["poses"])

    # --- resident inputs: one MPI replica per GPU (generated on device), packed once
    view = gen_view(H, W, P, c4["seed"], dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    packed = _lib.pack_planes(view) if args.kernel == "packed" else None
    torch.cuda.synchronize()
    pack_ms = (time.perf_counter() - t0) * 1e3
    if packed is not None:
        kernel_name, grid = _lib.route("render_packed", H, W, P, V)
    else:
        kernel_name, grid = _lib.route("render", V, H, W, P)

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
            _lib._call("mpiv_render_packed", packed, H, W, P, h_dev, n, o, _lib._stream(dev))
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

    # the short legs first (single view, configs 2 and 3, the notebook shape), so they do not
    # inherit a clock lowered by the sustained config-4 load (config 3 measured 0.75 ms after it
    # against 0.61-0.63 ms on a fresh clock, profiles/r03_sweep_few_depths_ab.txt)
    sv = single_view_leg(packed, H, W, P, host_homs(0, 1).to(dev), dev, stream) \
        if ("sv" in legs and packed is not None) else None
    c2 = config2_leg(dev, stream) if "c2" in legs else None
    torch.cuda.empty_cache()
    c3 = config3_leg(dev, stream) if "c3" in legs else None
    torch.cuda.empty_cache()
    nb = notebook_leg(dev, stream) if "nb" in legs else None
    torch.cuda.empty_cache()
    nout = guarded(netout_leg, dev, stream) if "netout" in legs else None
    torch.cuda.empty_cache()

    run(args.warmup, 0)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    mark("c4", dev)  # an empty marker kernel (phase tag of the rocprof summary), before the clock starts
    t0 = time.perf_counter()
    run(args.steps, args.warmup, events)
    torch.cuda.synchronize()
    barrier(world)
    mark("untimed", dev)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, world, dev)
    kern_ms_local = float(np.mean([a.elapsed_time(b) for a, b in events]))
    kern_all = all_ranks(kern_ms_local, world, dev)
    kern_ms = max(kern_all)

    # --- after the timed region: the last timed launch's first frame against a one-view
    # launch of the same pose (bit-exact), the gather ceiling, the census
    extras = len(legs) > 1 or legs != ["c4"]
    last = args.warmup + args.steps - 1
    timed_frame_sha = one_sha = None
    peak_gbs = float("nan")
    gathers = None
    frame_checks = []
    if extras:
        one = torch.empty((1, H, W, 3), device=dev)
        idx = step_indices(last)
        for j in sorted({0, V // 2, V - 1}):
            h1 = _host.render_homographies(poses[idx[j]:idx[j] + 1], depths, K.expand(1, 3, 3), 1).to(dev)
            launch(h1, 1, one)
            frame_checks.append({"view": j, "pose": idx[j], "sha16": sha16(out[j]),
                                 "bit_exact": bool(torch.equal(out[j].view(torch.int32), one[0].view(torch.int32)))})
        timed_frame_sha = frame_checks[0]["sha16"]
        one_sha = timed_frame_sha if all(c["bit_exact"] for c in frame_checks) else None
        peak_gbs = gather_peak_gbs(dev, stream)
        # the texture path's real work in the timed launches: the counting build of the same
        # kernel (mpiv_render_packed_census) re-renders the timed steps and adds up the
        # 64-lane 16-B gather instructions its waves issue
        if packed is not None:
            census = torch.zeros(1, dtype=torch.int64, device=dev)
            try:
                for s_ in range(args.warmup, args.warmup + args.steps):
                    _lib._call("mpiv_render_packed_census", packed, H, W, P, host_homs(s_).to(dev), V, out, census,
                               _lib._stream(dev))
                gathers = int(census.item()) // args.steps
            except RuntimeError:  # this view count does not route to the rows kernel
                gathers = None

    mpix_total = world * args.steps * V * H * W / 1e6
    value = mpix_total / elapsed
    tap_bytes = V * P * H * W * 64            # four 16-B taps per plane-sample (one-row kernel)
    hbm_alg_bytes = V * (P * H * W * 16 + H * W * 12)  # every view reading its MPI once (§8d)
    gather_bytes = gathers * kWaveBytes if gathers else tap_bytes
    achieved = gather_bytes / (kern_ms * 1e-3) / 1e9
    pf = prof_fields(kernel_name, grid, hbm_alg_bytes, kern_ms, "c4")
    traffic = pf.get("traffic")

    cpu_frames, cpu_view = None, None
    if "cpu" in legs and world == 1 and rank == 0 and packed is not None:
        one = torch.empty((1, H, W, 3), device=dev)
        launch(host_homs(0, 1).to(dev), 1, one)
        torch.cuda.synchronize()
        cpu_frames = [one.cpu().numpy()]
        cpu_view = view.cpu()
    del out
    if packed is not None:
        del view, packed
    torch.cuda.empty_cache()

    u8 = None
    if "u8" in legs:
        u8 = guarded(u8_leg, dev, stream, V, host_homs(0, 1).to(dev), host_homs(0).to(dev))
    train = guarded(training_leg, dev, stream) if "train" in legs else None
    ranks = {"world_size_seen": world, "backend": backend, "per_rank_kernel_ms": [round(x, 4) for x in kern_all]}
    if world > 1:
        import torch.distributed as dist
        ranks["world_size_seen"] = dist.get_world_size()
        ranks["one_device_rehearsal"] = os.environ.get("MPIV_BENCH_ONE_DEVICE") == "1"

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded U[-1,1) rgb / U[0,1) alpha MPI generated on device; viewer-style 1000-pose sway path)",
            "config": {"workload": "BASELINE config 4: 128-plane 1024x1024 MPI, 1000-pose camera path, view-sharded",
                       "H": H, "W": W, "planes": P, "views_per_gpu_per_step": V, "kernel": args.kernel,
                       "parallelism": f"view-sharded x{world} (replicas, no data-path collective)",
                       "views_per_s": round(value / (H * W / 1e6), 2), "pack_ms_once": round(pack_ms, 2),
                       # the one-time pack folded in, amortised over the 1000-pose path: every rank packs
                       # its replica once (in parallel), then renders its n_path / world poses
                       "value_incl_pack": round(n_path * H * W / 1e6 / ((pack_ms + n_path / (world * V) * elapsed
                                                                          / args.steps * 1e3) * 1e-3), 2),
                       "value_incl_pack_def": "1000 poses x H*W / (pack_ms_once + 1000/(n_gpus*V) x ms_per_step)",
                       "build_id": _lib.load().mpiv_build_id().decode()},
            "ranks": ranks,
            "roofline": {
                "bound": "texture", "achieved": round(achieved, 1),
                "peak": round(peak_gbs, 1) if peak_gbs == peak_gbs else None, "unit": "GB/s",
                "frac": round(achieved / peak_gbs, 4) if peak_gbs == peak_gbs else None, "traffic": traffic,
                "kernel": kernel_name, "grid_workitems": grid, "kernel_ms_per_launch": round(kern_ms, 3),
                "alg_bytes_per_launch": gather_bytes,
                "alg_bytes_def": ("gather instructions the launch issues (counted live by the kernel's census build, "
                                  "mpiv_render_packed_census) x 64 lanes x 16 B" if gathers else
                                  "V*P*H*W*64: four 16-B bilinear taps per plane-sample through the vector-memory path"),
                "gathers_per_plane_sample": round(gathers * 64 / (V * P * H * W), 3) if gathers else 4.0,
                "alg_bytes_4tap": tap_bytes,
                "peak_def": "mpiv_probe_gather on this device: 16-B/lane buffer loads from an L1/L2-resident "
                            "window with the render's access shape -- a measured TA ceiling, not a spec peak "
                            "(MI355X_MICROARCH.md L2: 34.5-36.9 TB/s)",
                "hbm_alg_bytes_per_launch": hbm_alg_bytes,
                "hbm_traffic_frac": pf.get("traffic_frac"),
                "hbm_traffic_over_compulsory": round(traffic / (P * (H + 4) * (W + 4) * 16 + V * H * W * 12), 2)
                if traffic else None,
                "compulsory_def": "packed MPI read once + V frames written",
                "mpi_reuse_per_launch": round(hbm_alg_bytes / traffic, 1) if traffic else None,
                "rocprof": {k: v for k, v in pf.items() if k not in ("kernel", "grid_workitems")},
                "single_view": sv,
            },
            "timed_frame_check": {"frames": "views 0, V/2 and V-1 of the last timed launch, each vs a 1-view "
                                            "launch of its pose", "views": frame_checks,
                                  "sha16": timed_frame_sha, "bit_exact": timed_frame_sha == one_sha}
            if extras else None,
            "cpu_baseline": None,
            "config2": c2,
            "config3_psv": c3,
            "notebook": nb,
            "u8_texels": u8,
            "net_output_render": nout,
            "training_render_backward": train,
            "config5_plane_sharded": None,
        }
        if cpu_frames is not None:
            res["cpu_baseline"] = cpu_baseline(cpu_view, host_homs(0), args.cpu_seconds, cpu_frames)
    else:
        res = {}
    # the plane-sharded leg last, under the LineGuard at world > 1: every figure above is already in
    # `res`, so a hung exchange costs only this leg's field, never the headline
    guard = LineGuard(rank)
    if world > 1 and "c5" in legs:
        guard.arm(LEG_DEADLINE_S, res, "config5_plane_sharded")
    # (a Python-level failure is recorded by guarded(); one that only some ranks see leaves the others
    # in the exchange, which the guard's deadline ends)
    c5 = guarded(config5_leg, world, rank, dev, max(3, args.steps // 2), 1) if "c5" in legs else None
    if rank == 0:
        res["config5_plane_sharded"] = c5
        guard.emit(res)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    guard.disarm()


if __name__ == "__main__":
    main()

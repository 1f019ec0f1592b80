"""Notebook-shape training step (224x224, 10 planes): per-step host time distribution with and without
Python's cyclic GC, and the device span of 50 back-to-back steps.  Probe only (GPU box)."""
import gc
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import configs  # noqa: E402

dev = torch.device("cuda:0")
N, P = 224, 10
f = configs.focal_from_fov(N)
K = configs.f32(configs.intrinsics_matrix(f, f, N / 2.0, N / 2.0)).to(dev)[None]
pose = configs.f32(configs.pose_from(configs.rot_y(1.0), (0.05, -0.02, 0.03))).to(dev)[None]
planes = configs.f32(mv.inv_depths(1, 100, P)).to(dev)
leaf = configs.synthetic_mpi(1, N, N, P, 9).to(dev).requires_grad_(True)
dout = torch.rand((1, N, N, 3), device=dev)


def step():
    mv.mpi_render_view_torch(leaf, pose, planes, K).backward(dout)
    leaf.grad = None


def host_dist(k=400):
    ts = []
    for _ in range(k):
        t = time.perf_counter()
        step()
        ts.append((time.perf_counter() - t) * 1e6)
    torch.cuda.synchronize()
    ts.sort()
    return {"p50": round(ts[len(ts) // 2], 1), "p90": round(ts[int(len(ts) * 0.9)], 1),
            "max": round(ts[-1], 1), "mean": round(statistics.mean(ts), 1)}


def span(n=50, reps=5):
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            step()
        b.record()
        torch.cuda.synchronize()
        out.append(round(a.elapsed_time(b) / n * 1e3, 1))
    return out


for _ in range(50):
    step()
res = {"gc_on": host_dist(), "span_us_gc_on": span()}
gc.disable()
res.update({"gc_off": host_dist(), "span_us_gc_off": span()})
gc.enable()
print(json.dumps(res))

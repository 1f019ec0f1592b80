"""Notebook-shape training step: host time per step (p50 over windows of 100 steps) across 3000 steps from
a cold start, and device spans of 50 steps at the end -- how long the host path takes to reach its steady
rate.  Probe only (GPU box)."""
import json
import os
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


wins = []
for w in range(30):
    ts = []
    for _ in range(100):
        t = time.perf_counter()
        step()
        ts.append((time.perf_counter() - t) * 1e6)
    ts.sort()
    wins.append(round(ts[50], 1))
torch.cuda.synchronize()
spans = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        step()
    b.record()
    torch.cuda.synchronize()
    spans.append(round(a.elapsed_time(b) / 50 * 1e3, 1))
print(json.dumps({"p50_per_100_steps_us": wins, "span_us": spans}))

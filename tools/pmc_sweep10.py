#!/usr/bin/env python3
"""Config-3 sources swept into D = inv_depths(1, 100, D) planes through mpiv_plane_sweep (the raw
route), a few launches, for rocprofv3 --pmc passes (tools/pmc_sweep10.sh).

    python tools/pmc_sweep10.py [--D 10] [--direct -1|0|1] [--iters 5]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--D", type=int, default=10)
ap.add_argument("--direct", type=int, default=-1)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
_lib.set_debug(sweep_direct=a.direct)
dev = torch.device("cuda:0")
c = configs.config3()
S, H, W, D = c["S"], c["H"], c["W"], a.D
img = torch.rand((S, H, W, 3), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
K = configs.f32([c["K"]] * S)
ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
ki, proj = ki.to(dev), proj.to(dev)
d = configs.f32(configs.inv_depths(1, 100, D)).to(dev)
out = torch.empty((S, H, W, D * 3), device=dev)
for _ in range(a.iters):
    _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, d, D, H, W, out, _lib._stream(dev))
torch.cuda.synchronize()
print("done", D, a.direct)

#!/usr/bin/env python3
"""Run the render backward at the config-4 size a few times (for rocprofv3 --pmc passes):
    python tools/pmc_bwd.py [--iters 2] [--cfg config4]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("--cfg", default="config4")
a = ap.parse_args()
dev = torch.device("cuda:0")
c = getattr(configs, a.cfg)()
H, W, P = c["H"], c["W"], c["P"]
g = torch.Generator(device=dev).manual_seed(0)
mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
homs = _host.render_homographies(configs.f32(c["poses"][:1]), configs.f32(c["depths"]), configs.f32([c["K"]]), 1)
dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
for _ in range(a.iters):
    _lib.render_backward(mpi, homs, dout)
torch.cuda.synchronize()

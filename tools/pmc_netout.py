#!/usr/bin/env python3
"""Run render_netout_kernel (bench.py netout_leg's case: config-2 size, pose 5) a few times for
rocprofv3 --pmc passes:  python tools/pmc_netout.py [--geo 821] [--iters 3]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--geo", type=int, default=0)
a = ap.parse_args()
dev = torch.device("cuda:0")
c = configs.config2()
H, W, P = c["H"], c["W"], c["P"]
g = torch.Generator(device=dev).manual_seed(c["seed"])
pred = torch.rand((1, 2 * P + 3, H, W), generator=g, device=dev) * 2 - 1
fg = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
homs = _host.render_homographies(configs.f32(c["poses"][5:6]), configs.f32(c["depths"]), configs.f32([c["K"]]), 1).to(dev)
out = torch.empty((1, H, W, 3), device=dev)
if a.geo:
    _lib.set_debug(netout_geo=a.geo)
for _ in range(a.iters):
    _lib._call("mpiv_render_net_output", pred, _lib._strides(pred), fg, _lib._strides(fg), 1, H, W, P, homs, out,
               _lib._stream(dev))
torch.cuda.synchronize()

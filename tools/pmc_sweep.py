#!/usr/bin/env python3
"""Run the config-3 plane sweep kernel a few times (for rocprofv3 --pmc passes).

    python tools/pmc_sweep.py [--store lds|tile|0|1|2] [--iters 3]

lds = the default LDS-staged kernel, pixlane = the pixel-per-lane LDS kernel, tile = the tile kernel, 0/1/2 = the grouped
kernel's store modes.
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--store", default="lds")
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
if a.store == "pixlane":
    _lib.load().mpiv_debug_set(b"sweep_dlane", 0)
elif a.store == "tile":
    _lib.load().mpiv_debug_set(b"sweep_tile", 1)
elif a.store != "lds":
    _lib.load().mpiv_debug_set(b"sweep_store", int(a.store))
dev = torch.device("cuda:0")
c = configs.config3()
S, H, W, D = c["S"], c["H"], c["W"], c["D"]
img = torch.rand((S, H, W, 3), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
K = configs.f32([c["K"]] * S)
ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
ki, proj = ki.to(dev), proj.to(dev)
d = configs.f32(c["depths"]).to(dev)
out = torch.empty((S, H, W, D * 3), device=dev)
img4 = _lib.pad_texels(img)
for _ in range(a.iters):
    _lib._call("mpiv_plane_sweep_padded", img4, S, H, W, 3, ki, proj, d, D, H, W, out, _lib._stream(dev))
torch.cuda.synchronize()
print("done", a.store)

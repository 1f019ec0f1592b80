#!/usr/bin/env python3
"""Run one render-kernel variant a few times (for rocprofv3 --pmc passes).

    python tools/pmc_render.py --variant mv|direct|lds --views 8 --iters 3

direct = the default direct-gather kernel, pair = pixel pairs sharing taps,
mv = the multi-view LDS kernel (debug option render_mv=1), lds = the single-view LDS
variant; chunk<N> = mpiv_render on the reference [1,H,W,P,4] layout with debug option
render_chunk=N (render_chunk.hip), native = the same layout, one pixel per lane.
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variant", default="mv")
ap.add_argument("--views", type=int, default=8)
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
if a.variant == "mv":
    _lib.load().mpiv_debug_set(b"render_mv", 1)
if a.variant == "pair":  # pixel pairs sharing taps (render_pair_kernel, A/B)
    _lib.load().mpiv_debug_set(b"render_pair", 1)
dev = torch.device("cuda:0")
c = configs.config4()
H, W, P, V = c["H"], c["W"], c["P"], a.views
g = torch.Generator(device=dev).manual_seed(0)
if a.variant.startswith("chunk") or a.variant == "native":
    _lib.load().mpiv_debug_set(b"render_chunk", int(a.variant[5:]) if a.variant != "native" else -1)
    mpi = torch.rand((V, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c["poses"][:V]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]] * V), V).to(dev)
    out = torch.empty((V, H, W, 3), device=dev)
    for _ in range(a.iters):
        _lib._call("mpiv_render", mpi, _lib._strides(mpi), V, H, W, P, homs, out, _lib._stream(dev))
    torch.cuda.synchronize()
    print("done", a.variant, V)
    sys.exit(0)
packed = torch.zeros(_lib.packed_shape(H, W, P), device=dev)
packed[:, 2:2 + H, 2:2 + W].uniform_(generator=g)
homs = _host.render_homographies(configs.f32(c["poses"][:V]), configs.f32(c["depths"]),
                                 configs.f32([c["K"]] * V), V).to(dev)
out = torch.empty((V, H, W, 3), device=dev)
name = "mpiv_render_packed_lds" if a.variant == "lds" else "mpiv_render_packed"
for _ in range(a.iters):
    _lib._call(name, packed, H, W, P, homs, V, out, _lib._stream(dev))
torch.cuda.synchronize()
print("done", a.variant, V)

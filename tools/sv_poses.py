#!/usr/bin/env python3
"""Single-view render time along the config-4 camera path, per kernel variant
(A/B for the packed single-view routing): python tools/sv_poses.py [--poses 0,125,...]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--poses", default="0,125,250,375,500,625,750,875")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
c = configs.config4()
H, W, P = c["H"], c["W"], c["P"]
g = torch.Generator(device=dev).manual_seed(0)
view = torch.rand((H, W, P, 4), generator=g, device=dev)
packed = _lib.pack_planes(view)
out = torch.empty((1, H, W, 3), device=dev)
stream = torch.cuda.current_stream(dev)
for k in [int(x) for x in a.poses.split(",")]:
    h = _host.render_homographies(configs.f32([c["poses"][k]]), configs.f32(c["depths"]),
                                  configs.f32([c["K"]]), 1).to(dev)
    row = {"pose": k}
    for name, opts in (("default", {}), ("direct", {"render_tile": -1}), ("ring4", {"render_ring": 4}),
                       ("ring8", {"render_ring": 8}), ("rows4", {"render_tile": 4}), ("rows8", {"render_tile": 8}),
                       ("rows16", {"render_tile": 16}), ("lds", None)):
        fn = (lambda: _lib._call("mpiv_render_packed_lds", packed, H, W, P, h, 1, out, _lib._stream(dev))) \
            if opts is None else (lambda: _lib._call("mpiv_render_packed", packed, H, W, P, h, 1, out, _lib._stream(dev)))
        with _lib.debug(**(opts or {})):
            fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
            for s, e in ev:
                s.record(stream)
                fn()
                e.record(stream)
            torch.cuda.synchronize()
        row[name] = round(float(np.median([s.elapsed_time(e) for s, e in ev])), 4)
    print(json.dumps(row), flush=True)

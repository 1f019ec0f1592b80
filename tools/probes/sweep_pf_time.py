#!/usr/bin/env python3
"""Timing probe: the LDS-staged sweep as one block per tile (sweep_pf=-1) or resident blocks with
the next tile prefetched (sweep_pf=1), config 3's sources at D = 64 and the notebook's D = 10;
volumes compared bit for bit between the two."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    c = configs.config3()
    S, H, W = c["S"], c["H"], c["W"]
    g = torch.Generator(device=dev).manual_seed(c["seed"])
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    pose = configs.f32(c["poses"])
    ki, proj = _host.psv_matrices(K, K, pose)
    ki, proj = ki.to(dev), proj.to(dev)
    lib = os.path.basename(os.environ.get("MPIV_LIB", "libmpiv.so"))
    for D, SS in ((64, S), (10, 4)):
        dd = configs.f32(list(c["depths"]) if D == 64 else configs.inv_depths(1, 100, D)).to(dev)
        im = img[:SS]
        outs = {}
        for rep in range(2):
            for pf in [int(x) for x in os.environ.get("PFS", "-1,1").split(",")]:
                optname = os.environ.get("OPT", "sweep_pf")
                out = torch.empty((SS, H, W, D * 3), device=dev)
                fn = lambda: _lib._call("mpiv_plane_sweep", im, _lib._strides(im), SS, H, W, 3, ki, proj, dd,  # noqa: E731
                                        D, H, W, out, _lib._stream(dev))
                with _lib.debug(**{optname: pf}):
                    for _ in range(10):
                        fn()
                    torch.cuda.synchronize()
                    s = torch.cuda.current_stream()
                    ts = []
                    for _ in range(7):
                        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record(s)
                        for _ in range(10):
                            fn()
                        b.record(s)
                        b.synchronize()
                        ts.append(a.elapsed_time(b) / 10)
                    ts.sort()
                route = _lib.route("plane_sweep", SS, H, W, 3, D, H, W)[0] if pf == 0 else pf
                outs[pf] = out
                print(json.dumps({"lib": lib, "D": D, "S": SS, "opt": optname, "pf": pf, "rep": rep, "route": route, "ms": round(ts[3], 4),
                                  "min": round(ts[0], 4)}), flush=True)
            if len(outs) == 2:
                same = bool(torch.equal(outs[-1].view(torch.int32), outs[1].view(torch.int32)))
                print(json.dumps({"lib": lib, "D": D, "same": same}), flush=True)
            outs.clear()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Timing probe for render_netout_kernel under the loaded library (MPIV_LIB selects a probe
build): median of back-to-back launch spans for each geometry, frames compared with the two-step
assemble + render (a timing-only build may differ; its frames are reported, not asserted)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(c["seed"])
    pred = torch.rand((1, 2 * P + 3, H, W), generator=g, device=dev) * 2 - 1
    fg = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    lib = os.path.basename(os.environ.get("MPIV_LIB", "libmpiv.so"))
    geos = [int(x) for x in os.environ.get("GEOS", "821,1821").split(",")]
    # OPTS: extra debug options to A/B, "name=v;name=v" alternatives (e.g. "netout_fg3=0;netout_fg3=1")
    alts = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",") if kv)
            for a in os.environ.get("OPTS", "").split(";")] or [{}]
    for pose in (5, 20):
        homs = _host.render_homographies(configs.f32(c["poses"][pose:pose + 1]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]]), 1).to(dev)
        out = torch.empty((1, H, W, 3), device=dev)
        two = _lib.render(_lib.assemble_mpi(pred, fg, P), homs)
        fn = lambda: _lib._call("mpiv_render_net_output", pred, _lib._strides(pred), fg, _lib._strides(fg), 1,  # noqa: E731
                                H, W, P, homs, out, _lib._stream(dev))
        for rep in range(2):
            for geo, alt in [(g_, a_) for g_ in geos for a_ in alts]:
                with _lib.debug(netout_geo=geo, **alt):
                    for _ in range(20):
                        fn()
                    torch.cuda.synchronize()
                    s = torch.cuda.current_stream()
                    ts = []
                    for _ in range(7):
                        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record(s)
                        for _ in range(20):
                            fn()
                        b.record(s)
                        b.synchronize()
                        ts.append(a.elapsed_time(b) / 20)
                    ts.sort()
                    same = bool(torch.equal(out.view(torch.int32), two.view(torch.int32)))
                    print(json.dumps({"lib": lib, "pose": pose, "geo": geo, "opts": alt, "rep": rep, "ms": round(ts[3], 4),
                                      "min": round(ts[0], 4), "same": same}), flush=True)


if __name__ == "__main__":
    main()

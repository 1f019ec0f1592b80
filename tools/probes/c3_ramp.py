#!/usr/bin/env python3
"""Per-launch times of the config-3 sweep after an idle gap: the shape of the slow start the bench's
config-3 leg sees (kernel_ms_first_last_third).  Runs: a host gap of 0 / 50 / 200 ms (synchronised,
then idle) before 60 back-to-back launches, each bracketed by its own events."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    c = configs.config3()
    S, H, W, D = c["S"], c["H"], c["W"], c["D"]
    g = torch.Generator(device=dev).manual_seed(c["seed"])
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
    ki, proj = ki.to(dev), proj.to(dev)
    dd = configs.f32(list(c["depths"])).to(dev)
    out = torch.empty((S, H, W, D * 3), device=dev)
    s = torch.cuda.current_stream()
    fn = lambda: _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, dd, D, H, W,  # noqa: E731
                            out, _lib._stream(dev))
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    for gap in (0.0, 0.05, 0.2, 0.0):
        time.sleep(gap)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(61)]
        ev[0].record(s)
        for i in range(60):
            fn()
            ev[i + 1].record(s)
        ev[-1].synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(60)]
        print(json.dumps({"gap_s": gap, "first10": [round(x, 3) for x in ms[:10]],
                          "mean_thirds": [round(sum(ms[k:k + 20]) / 20, 4) for k in (0, 20, 40)],
                          "mean": round(sum(ms) / 60, 4)}), flush=True)
        # a 3-GB read like the bench's bit check, then the same sequence
    same = bool(torch.equal(out.view(torch.int32), out.view(torch.int32)))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(61)]
    ev[0].record(s)
    for i in range(60):
        fn()
        ev[i + 1].record(s)
    ev[-1].synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(60)]
    print(json.dumps({"after": "torch.equal of the volume", "ok": same, "first10": [round(x, 3) for x in ms[:10]],
                      "mean_thirds": [round(sum(ms[k:k + 20]) / 20, 4) for k in (0, 20, 40)]}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Timing probe for the config-4 render backward (with checkpoints) under the loaded library (MPIV_LIB
selects a probe build): back-to-back spans after a warm-up, and the gradient's sha16 for a bit-identity
check across builds."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(0)
    mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c["poses"][100:101]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1).to(dev)
    dout = torch.rand((1, H, W, 3), generator=torch.Generator(device=dev).manual_seed(1), device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
    got = fn()
    sha = hashlib.sha256(got.cpu().numpy().tobytes()).hexdigest()[:16]
    lib = os.path.basename(os.environ.get("MPIV_LIB", "libmpiv.so"))
    for rep in range(3):
        for _ in range(30):
            fn()
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(20):
            fn()
        b.record(s)
        b.synchronize()
        print(json.dumps({"lib": lib, "rep": rep, "backward_ms": round(a.elapsed_time(b) / 20, 4), "grad_sha16": sha}),
              flush=True)


if __name__ == "__main__":
    main()

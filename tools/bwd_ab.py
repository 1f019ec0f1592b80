"""Render-backward A/B on the GPU (config 4, one view with checkpoints): the production
gather against the variants selected by bwd_gather=k, bit-identical gradients required.
    python tools/bwd_ab.py [k ...]      (default: 0 3)"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402


def main():
    variants = [int(a) for a in sys.argv[1:]] or [0, 3]
    dev = torch.device("cuda:0")
    c4 = configs.config4()
    H, W, P = c4["H"], c4["W"], c4["P"]
    g = torch.Generator(device=dev).manual_seed(7)
    mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c4["poses"][100:101]), configs.f32(c4["depths"]),
                                     configs.f32([c4["K"]]), 1).to(dev)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    ref = None
    for rep in range(2):
        for v in variants:
            _lib.set_debug(bwd_gather=v)
            out = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
            flag = int(ws[_lib.bwd_flag_offset(H, W, P):][:4].view(torch.int32).item())
            if ref is None:
                ref = out.clone()
            same = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            for _ in range(3):
                _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for a, b in ev:
                a.record()
                _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
                b.record()
            torch.cuda.synchronize()
            ms = sorted(a.elapsed_time(b) for a, b in ev)
            ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev2:  # without checkpoints (the backward recomputes them)
                a.record()
                _lib.render_backward(mpi, homs, dout, workspace=ws)
                b.record()
            torch.cuda.synchronize()
            ms2 = sorted(a.elapsed_time(b) for a, b in ev2)
            nock_same = bool(torch.equal(_lib.render_backward(mpi, homs, dout, workspace=ws).view(torch.int32),
                                         out.view(torch.int32)))
            _lib.reset_debug()
            sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
            print(json.dumps({"rep": rep, "bwd_gather": v, "median_ms": round(ms[len(ms) // 2], 4),
                              "min_ms": round(ms[0], 4), "bit_identical_in_process": same, "grad_sha16": sha,
                              "no_ckpt_median_ms": round(ms2[len(ms2) // 2], 4), "no_ckpt_bit_identical": nock_same,
                              "fallback_flag": flag}), flush=True)


if __name__ == "__main__":
    main()

"""Folded vs unfolded render-backward schedule (round 6) at config-2 and config-4 sizes: ms per call
(HIP events, back to back) and the fallback flag after a call.  Probe only (GPU box)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for name, c in (("c2", configs.config2()), ("c4", configs.config4())):
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(7)
    mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c["poses"][5:6]), configs.f32(c["depths"]), configs.f32([c["K"]]),
                                     1).to(dev)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    _, ck = _lib.render_train(mpi, homs)
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    for unfold in (0, 1, 0):
        _lib.set_debug(bwd_unfold=unfold)
        fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck, check=False)  # noqa: E731
        for _ in range(5):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            fn()
        b.record()
        torch.cuda.synchronize()
        off = _lib.bwd_flag_offset(H, W, P)
        out[f"{name}_unfold{unfold}"] = {"ms": round(a.elapsed_time(b) / 10, 4),
                                         "flags": ws[off:off + 40].view(torch.int32).tolist()}
        _lib.reset_debug()
    del mpi, ws, ck
    torch.cuda.empty_cache()
print(json.dumps(out))

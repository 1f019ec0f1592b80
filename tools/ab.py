#!/usr/bin/env python3
"""Kernel A/B timings on the GPU box (round 3): each experiment times the production
entry point under a set of libmpiv debug options, alternating the variants twice so a
drifting clock shows up as disagreement between the two passes.  One JSON line per
measurement (median of --iters launches, HIP events on the launch stream).

    python tools/ab.py --only chunk,train,bwd,sweep,sweep10,u8
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from mpi_vision_amd import _host, _lib, configs  # noqa: E402

PEAK = 8000.0


def timed(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts), min(ts)


def span(fn, iters, warmup=3):
    """Back-to-back launches: device time of `iters` launches between two events / iters (a
    write-heavy kernel's drain then lands in the next launch, as in bench.py's legs)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / iters


def run(name, variants, fn, alg, iters, passes=2):
    for p in range(passes):
        for label, opts in variants:
            with _lib.debug(**opts):
                ms, mn = timed(fn, iters)
                b2b = span(fn, iters)
            print(json.dumps({"exp": name, "variant": label, "pass": p, "ms": round(ms, 4), "ms_min": round(mn, 4),
                              "ms_b2b": round(b2b, 4), "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK, 4)}), flush=True)


def c4_mpi(dev, B=1):
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(0)
    mpi = torch.rand((B, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c["poses"][100:100 + B]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]] * B), B).to(dev)
    return mpi, homs, H, W, P


ROWS = [("rows1", {"chunk_rows": 1}), ("rows2", {"chunk_rows": 2}), ("rows4", {"chunk_rows": 4})]


def chunk(dev, it):
    mpi, homs, H, W, P = c4_mpi(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out, _lib._stream(dev))  # noqa: E731
    run("c4 in-place render (render_chunk_kernel), 1 view", ROWS, fn, P * H * W * 16 + H * W * 12, it)


def train(dev, it):
    mpi, homs, H, W, P = c4_mpi(dev)
    fn = lambda: _lib.render_train(mpi, homs)  # noqa: E731
    run("c4 training forward (frame + checkpoints), 1 view", ROWS, fn, P * H * W * 16 + H * W * 12, it)


def bwd(dev, it):
    mpi, homs, H, W, P = c4_mpi(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
    run("c4 render backward with checkpoints, 1 view", ROWS, fn, 2 * P * H * W * 16 + H * W * 12, it)


def bwdgrp(dev, it):
    """The backward in plane groups of 8 / 16 / 32 planes vs one group: a group's d samples (8 planes:
    134 MB at config 4) fit the 256-MB Infinity Cache between its chain and its gather."""
    mpi, homs, H, W, P = c4_mpi(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    _, ck = _lib.render_train(mpi, homs)
    ref = None
    for p in range(2):
        for grp, ov in ((0, 0), (0, 1), (16, 1), (32, 0), (64, 1)):
            with _lib.debug(bwd_group=grp, bwd_overlap=ov):
                ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
                fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
                got = fn()
                if ref is None:
                    ref = got.clone()
                same = bool(torch.equal(got.view(torch.int32), ref.view(torch.int32)))
                ms, mn = timed(fn, it)
                b2b = span(fn, it)
                print(json.dumps({"exp": "c4 backward plane groups", "variant": f"group{grp}_overlap{ov}", "pass": p, "ms": round(ms, 4),
                                  "ms_min": round(mn, 4), "ms_b2b": round(b2b, 4), "ws_GB": round(ws.numel() / 1e9, 3),
                                  "same": same}), flush=True)
                del ws, got
                torch.cuda.empty_cache()


STRIP = [("rows64x1", {"chunk_strip": 0}), ("strip8x16", {"chunk_strip": 1})]
STRIPS = [("strip8x16", {"chunk_strip": 1}), ("strip8x8", {"chunk_strip": 2}), ("strip8x8_nt3", {"chunk_strip": 3}),
          ("strip8x16_nt3", {"chunk_strip": 4})]


def strips(dev, it):
    """Round 4: strip shapes of render_chunk_strip_kernel (in-place render, training forward)."""
    mpi, homs, H, W, P = c4_mpi(dev)
    ref = None
    for label, opts in STRIPS:
        with _lib.debug(**opts):
            f, ck = _lib.render_train(mpi, homs)
        if ref is None:
            ref = (f, ck)
        print(json.dumps({"exp": "strips bit identity", "variant": label,
                          "frames": bool(torch.equal(f.view(torch.int32), ref[0].view(torch.int32))),
                          "ckpts": bool(torch.equal(ck.view(torch.int32), ref[1].view(torch.int32)))}), flush=True)
    del ref, f, ck
    out = torch.empty((1, H, W, 3), device=dev)
    fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out, _lib._stream(dev))  # noqa: E731
    run("c4 in-place render, 1 view", STRIPS, fn, P * H * W * 16 + H * W * 12, it, passes=2)
    fn = lambda: _lib.render_train(mpi, homs)  # noqa: E731
    run("c4 training forward (frame + checkpoints), 1 view", STRIPS, fn, P * H * W * 16 + H * W * 12, it, passes=2)
    g = torch.Generator(device=dev).manual_seed(1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    chains = [("chain64x1", {"chunk_strip": 0}), ("chain8x16", {"chunk_strip": 1}), ("chain8x8", {"chunk_strip": 2})]
    grads = []
    for label, opts in chains:
        with _lib.debug(**opts):
            grads.append(_lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck, check=True))
    print(json.dumps({"exp": "chain strips bit identity", "grads": [bool(torch.equal(x.view(torch.int32),
                                                                                      grads[0].view(torch.int32)))
                                                                     for x in grads]}), flush=True)
    del grads
    fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
    run("c4 render backward with checkpoints, 1 view", chains, fn, 2 * P * H * W * 16 + H * W * 12, it, passes=2)


def striph(dev, it):
    """Round 5: render_chunk_strip_kernel<16, 2> with its homographies in LDS (3 blocks per CU) or read
    through the caches (chunk_strip=5: a fourth block per CU); frames compared bit for bit."""
    mpi, homs, H, W, P = c4_mpi(dev)
    variants = [("strip_hlds", {"chunk_strip": 1}), ("strip_hglobal", {"chunk_strip": 5})]
    out = torch.empty((1, H, W, 3), device=dev)
    fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out, _lib._stream(dev))  # noqa: E731
    frames = []
    for label, opts in variants:
        with _lib.debug(**opts):
            fn()
            torch.cuda.synchronize()
            frames.append(out.clone())
    print(json.dumps({"exp": "striph bit identity", "frames": bool(torch.equal(frames[0].view(torch.int32),
                                                                                frames[1].view(torch.int32)))}), flush=True)
    for _ in range(60):
        fn()
    run("c4 in-place render, 1 view", variants, fn, P * H * W * 16 + H * W * 12, it, passes=3)


def strip(dev, it):
    """Round 4: render_chunk_strip_kernel (8 x 8 strips, vertical tap reuse) vs the 64 x 1
    wave rows, in-place render and training forward; frames and checkpoints compared bit for bit."""
    mpi, homs, H, W, P = c4_mpi(dev)
    res = {}
    for label, opts in STRIP:
        with _lib.debug(**opts):
            res[label] = _lib.render_train(mpi, homs)
    (fa, ca), (fb, cb) = res.values()
    print(json.dumps({"exp": "strip bit identity", "frames": bool(torch.equal(fa.view(torch.int32), fb.view(torch.int32))),
                      "ckpts": bool(torch.equal(ca.view(torch.int32), cb.view(torch.int32)))}), flush=True)
    del res, fa, fb, ca, cb
    out = torch.empty((1, H, W, 3), device=dev)
    fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out, _lib._stream(dev))  # noqa: E731
    run("c4 in-place render, 1 view", STRIP, fn, P * H * W * 16 + H * W * 12, it, passes=3)
    fn = lambda: _lib.render_train(mpi, homs)  # noqa: E731
    run("c4 training forward (frame + checkpoints), 1 view", STRIP, fn, P * H * W * 16 + H * W * 12, it, passes=3)
    g = torch.Generator(device=dev).manual_seed(1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    grads = []
    for label, opts in STRIP:
        with _lib.debug(**opts):
            grads.append(_lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck, check=True))
    print(json.dumps({"exp": "strip chain bit identity", "grads": bool(torch.equal(grads[0].view(torch.int32),
                                                                                    grads[1].view(torch.int32)))}),
          flush=True)
    del grads
    fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
    run("c4 render backward with checkpoints, 1 view", STRIP, fn, 2 * P * H * W * 16 + H * W * 12, it, passes=3)


U8F = [("u8_flight2", {"u8_flight": 2}), ("u8_flight4", {"u8_flight": 4}), ("u8_flight8", {"u8_flight": 8})]


def u8f(dev, it):
    """Round 4: the u8 render (vertical reuse, 4 rows) with 2 vs 4 rows in flight, 1 and 125 views."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    pk = _lib.synth_mpi_packed_u8(c["seed"], H, W, 0, P, dev)
    for V, pose0, iters in ((1, 100, it), (125, 0, 3)):
        homs = _host.render_homographies(configs.f32(c["poses"][pose0:pose0 + V]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]] * V), V).to(dev)
        out = torch.empty((V, H, W, 3), device=dev)
        outs = []
        for label, opts in U8F:
            with _lib.debug(**opts):
                _lib._call("mpiv_render_packed_u8", pk, H, W, P, homs, V, out, _lib._stream(dev))
            outs.append(out.clone())
        import hashlib
        print(json.dumps({"exp": f"u8 flight bit identity, {V} views",
                          "same": [bool(torch.equal(o.view(torch.int32), outs[0].view(torch.int32))) for o in outs],
                          "sha16": hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest()[:16]}), flush=True)
        del outs
        fn = lambda: _lib._call("mpiv_render_packed_u8", pk, H, W, P, homs, V, out, _lib._stream(dev))  # noqa: E731
        run(f"u8 render, {V} views", U8F, fn, V * (P * H * W * 4 + H * W * 12), iters, passes=2)
        del out
        torch.cuda.empty_cache()


FLIGHT = [("flight2", {}), ("flight4", {"chunk_flight": 4})]


def chunkf(dev, it):
    mpi, homs, H, W, P = c4_mpi(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out, _lib._stream(dev))  # noqa: E731
    run("c4 in-place render (render_chunk_kernel), 1 view", FLIGHT, fn, P * H * W * 16 + H * W * 12, it)
    fn2 = lambda: _lib.render_train(mpi, homs)  # noqa: E731
    run("c4 training forward (frame + checkpoints), 1 view", FLIGHT, fn2, P * H * W * 16 + H * W * 12, it)


SWROWS = [("rows4", {}), ("rows6", {"sweep_rows": 6}), ("rows8", {"sweep_rows": 8})]


def sweep(dev, it):
    c = configs.config3()
    S, H, W = c["S"], c["H"], c["W"]
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
    ki, proj = ki.to(dev), proj.to(dev)
    for D in (64, 10):
        d = configs.f32(configs.inv_depths(1, 100, D)).to(dev)
        out = torch.empty((S, H, W, D * 3), device=dev)
        fn = lambda: _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, d, D, H, W,  # noqa: E731
                                out, _lib._stream(dev))
        run(f"c3 sources -> {D} planes (mpiv_plane_sweep)", SWROWS, fn, S * H * W * 12 + S * D * H * W * 12, it)
        del out


GATHER = [("block", {}), ("ws", {"bwd_gather": 2})]


def bwdg(dev, it):
    mpi, homs, H, W, P = c4_mpi(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    ref = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
    import hashlib
    print(json.dumps({"exp": "bwd gradient sha16", "sha16": hashlib.sha256(ref.cpu().numpy().tobytes()).hexdigest()[:16]}))
    flag_off = _lib.bwd_flag_offset(H, W, P)
    for label, opts in GATHER:
        with _lib.debug(**opts):
            got = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
            flag = int(ws[flag_off:flag_off + 4].view(torch.int32).item())
        print(json.dumps({"exp": "bwd gather parity", "variant": label, "bit_identical":
                          bool(torch.equal(got.view(torch.int32), ref.view(torch.int32))), "fallback_flag": flag}))
    fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
    run("c4 render backward with checkpoints, 1 view", GATHER, fn, 2 * P * H * W * 16 + H * W * 12, it)


def swband(dev, it):
    """The LDS-staged sweep with one box per 4-row tile (plane_sweep_dlane_kernel, sweep_band=0) against
    the band-walking ring kernel (plane_sweep_band_kernel, sweep_band=1): config-3 sources into 10 / 16 /
    64 depths (4 and 5 sources, as bench.py's legs), bit-identical volumes checked first."""
    c = configs.config3()
    S, H, W = c["S"], c["H"], c["W"]
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
    ki, proj = ki.to(dev), proj.to(dev)
    for D, Sx in ((10, 4), (16, 4), (64, 5)):
        d = configs.f32(configs.inv_depths(1, 100, D)).to(dev)
        out = torch.empty((Sx, H, W, D * 3), device=dev)
        im = img[:Sx]
        alg = Sx * H * W * 12 + Sx * D * H * W * 12
        raw = lambda: _lib._call("mpiv_plane_sweep", im, _lib._strides(im), Sx, H, W, 3, ki, proj, d, D, H, W,  # noqa: E731
                                 out, _lib._stream(dev))
        vols = []
        for b in (0, 1):
            with _lib.debug(sweep_band=b, sweep_direct=-1):
                out.zero_()
                raw()
                vols.append(out.clone())
        print(json.dumps({"exp": "sweep band bit-exact", "D": D,
                          "same": bool(torch.equal(vols[0].view(torch.int32), vols[1].view(torch.int32)))}), flush=True)
        del vols
        run(f"c3 sources ({Sx}) -> {D} planes", [("dlane", {"sweep_band": 0, "sweep_direct": -1}),
                                                ("band", {"sweep_band": 1, "sweep_direct": -1})], raw, alg, it)
        del out
        torch.cuda.empty_cache()


def sw10(dev, it):
    """Config-3 sources into few depths (the notebook dataset's 10 planes) through
    mpiv_plane_sweep: the direct depth-per-lane kernel (no LDS staging) against the LDS-staged
    one and the pixel-per-lane one (sweep_direct=1 / -1 / 2; automatic: direct for D <= 8)."""
    c = configs.config3()
    S, H, W = c["S"], c["H"], c["W"]
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
    ki, proj = ki.to(dev), proj.to(dev)
    for D in [int(v) for v in os.environ.get("SW_D", "6,10,16,32,64").split(",")]:
        d = configs.f32(configs.inv_depths(1, 100, D)).to(dev)
        out = torch.empty((S, H, W, D * 3), device=dev)
        alg = S * H * W * 12 + S * D * H * W * 12
        raw = lambda: _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, d, D, H, W,  # noqa: E731
                                 out, _lib._stream(dev))
        run(f"c3 sources -> {D} planes (mpiv_plane_sweep)", [("lds", {"sweep_direct": -1}), ("direct", {"sweep_direct": 1}),
                                                                 ("px", {"sweep_direct": 2}), ("px32", {"sweep_direct": 3})],
            raw, alg, it)
        del out


def c3(dev, it):
    """BASELINE config 3 through mpiv_plane_sweep (the default route), isolated and back to back."""
    c = configs.config3()
    S, H, W, D = c["S"], c["H"], c["W"], c["D"]
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
    ki, proj = ki.to(dev), proj.to(dev)
    d = configs.f32(c["depths"]).to(dev)
    out = torch.empty((S, H, W, D * 3), device=dev)
    fn = lambda: _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, d, D, H, W,  # noqa: E731
                            out, _lib._stream(dev))
    run("c3 (mpiv_plane_sweep)", [("default", {})], fn, S * H * W * 12 + S * D * H * W * 12, it)


VSD = [("auto", {}), ("r8d4", {"render_vshare": 3}), ("r6d3", {"render_vshare": 4}), ("r9d3", {"render_vshare": 5}),
       ("r4d4", {"render_vshare": 11})]


def vsd(dev, it):
    """The packed render's (rows, rows in flight) routing on config 4 (bench.py's camera-path
    views): 125, 8 and 1 views per launch, every shipped (R, D) choice."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(0)
    view = torch.rand((H, W, P, 4), generator=g, device=dev)
    packed = _lib.pack_planes(view)
    del view
    for V in (125, 8, 1):
        homs = _host.render_homographies(configs.f32(c["poses"][:V]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]] * V), V).to(dev)
        out = torch.empty((V, H, W, 3), device=dev)
        fn = lambda: _lib._call("mpiv_render_packed", packed, H, W, P, homs, V, out, _lib._stream(dev))  # noqa: E731
        run(f"c4 packed render, {V} views", VSD, fn, V * (P * H * W * 16 + H * W * 12), max(3, it // (1 + V // 8)))
        del out


def chunkpar(dev, it):
    """Diagnostic: the in-place render (render_chunk_kernel) with the camera-path homographies
    against the same launch with every plane given plane 63's homography (no parallax inside a
    chunk: each 8-lane group's taps share one 128-B line) -- the most any parallax-following lane
    mapping could gain."""
    mpi, homs, H, W, P = c4_mpi(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    flat = homs.view(1, P, 9)[:, 63:64].expand(1, P, 9).contiguous()
    for label, hh in (("camera", homs), ("no_parallax", flat)):
        fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, hh, out, _lib._stream(dev))  # noqa: E731
        run(f"c4 in-place render, 1 view, {label}", DEF, fn, P * H * W * 16 + H * W * 12, it)


DEF = [("default", {})]


def netout(dev, it):
    """render_netout_kernel (network output -> view, bench.py netout_leg's case) with 1 / 2 / 4 rows
    per work-item; every variant's frame is checked against the two-step assemble + render."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(c["seed"])
    pred = torch.rand((1, 2 * P + 3, H, W), generator=g, device=dev) * 2 - 1
    fg = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    for k in (5, 20):
        homs = _host.render_homographies(configs.f32(c["poses"][k:k + 1]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]]), 1).to(dev)
        out = torch.empty((1, H, W, 3), device=dev)
        fn = lambda: _lib._call("mpiv_render_net_output", pred, _lib._strides(pred), fg, _lib._strides(fg), 1,  # noqa: E731
                                H, W, P, homs, out, _lib._stream(dev))
        two = _lib.render(_lib.assemble_mpi(pred, fg, P), homs)
        variants = [(f"geo{gg}b{bb}", {"netout_geo": gg, "netout_buf": bb}) for gg in (811, 821, 822, 422) for bb in (0, 1)]
        for label, opts in variants:
            with _lib.debug(**opts):
                out.zero_()
                fn()
                torch.cuda.synchronize()
                print(json.dumps({"exp": "netout bit-exact", "pose": k, "variant": label,
                                  "same": bool(torch.equal(out.view(torch.int32), two.view(torch.int32)))}), flush=True)
        run(f"netout 1024x576x32, pose {k}", variants, fn, H * W * ((2 * P + 3) * 4 + 24), it)


def dflt(dev, it):
    """The default routes of the training path (in-place render, training forward, backward with
    checkpoints) -- for A/B across library builds (MPIV_LIB, tools/gpu_ab_any.sh)."""
    mpi, homs, H, W, P = c4_mpi(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out, _lib._stream(dev))  # noqa: E731
    run("c4 in-place render, 1 view", DEF, fn, P * H * W * 16 + H * W * 12, it)
    run("c4 training forward, 1 view", DEF, lambda: _lib.render_train(mpi, homs), P * H * W * 16 + H * W * 12, it)
    g = torch.Generator(device=dev).manual_seed(1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    ws = torch.empty(_lib.load().mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    _, ck = _lib.render_train(mpi, homs)
    got = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)
    import hashlib
    print(json.dumps({"exp": "bwd gradient sha16", "sha16": hashlib.sha256(got.cpu().numpy().tobytes()).hexdigest()[:16],
                      "frame_sha16": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]}))
    fn = lambda: _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck)  # noqa: E731
    run("c4 render backward with checkpoints, 1 view", DEF, fn, 2 * P * H * W * 16 + H * W * 12, it)


def same(dev, it):
    """Round 6: same-row tap reuse (render.hip SAME) on the stretched configs -- config 2 at 64 and 8
    views, config 5's plane shard (C, T) -- against the vertical reuse alone (render_same=-1), at the
    automatic (R, D) and the other shipped ones; frames compared bit for bit first."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(0)
    view = torch.rand((H, W, P, 4), generator=g, device=dev)
    packed = _lib.pack_planes(view)
    del view
    V2 = len(c["poses"])
    homs_all = _host.render_homographies(configs.f32(c["poses"]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]] * V2), V2).to(dev)
    for V in (V2, 8):
        homs = homs_all[:V].contiguous()
        out = torch.empty((V, H, W, 3), device=dev)
        fn = lambda: _lib._call("mpiv_render_packed", packed, H, W, P, homs, V, out, _lib._stream(dev))  # noqa: E731
        vs = [("off", {"render_same": -1}), ("same", {})]
        for r in (3, 4, 5, 11):
            vs += [(f"off_vs{r}", {"render_same": -1, "render_vshare": r}), (f"same_vs{r}", {"render_vshare": r})]
        frames = []
        for label, opts in vs:
            with _lib.debug(**opts):
                out.zero_()
                fn()
                frames.append(out.clone())
        print(json.dumps({"exp": f"same bit identity, c2 {V} views", "same": [bool(torch.equal(
            f.view(torch.int32), frames[0].view(torch.int32))) for f in frames]}), flush=True)
        del frames
        run(f"c2 packed render, {V} views", vs, fn, V * (P * H * W * 16 + H * W * 12), it)
        del out
    del packed
    c5c = configs.config5()
    H, W, P = c5c["H"], c5c["W"], c5c["P"]
    PL = P // 8
    packed = torch.zeros(_lib.packed_shape(H, W, PL), device=dev)
    packed[:, 2:2 + H, 2:2 + W].uniform_(generator=g)
    homs = _host.render_homographies(configs.f32(c5c["poses"]), configs.f32(c5c["depths"]), configs.f32([c5c["K"]]),
                                     1)[:, :PL].contiguous().to(dev)
    ct = torch.empty((1, H, W, 4), device=dev)
    fn = lambda: _lib.render_packed_ct(packed, homs, back=True, out=ct)  # noqa: E731
    vs = [("off", {"render_same": -1}), ("same", {}), ("off_vs3", {"render_same": -1, "render_vshare": 3}),
          ("same_vs3", {"render_vshare": 3}), ("off_vs4", {"render_same": -1, "render_vshare": 4}),
          ("same_vs4", {"render_vshare": 4})]
    frames = []
    for label, opts in vs:
        with _lib.debug(**opts):
            ct.zero_()
            fn()
            frames.append(ct.clone())
    print(json.dumps({"exp": "same bit identity, c5 shard", "same": [bool(torch.equal(
        f.view(torch.int32), frames[0].view(torch.int32))) for f in frames]}), flush=True)
    del frames
    run(f"c5 plane shard {PL} of {P}, (C,T)", vs, fn, PL * H * W * 16 + H * W * 16, it)


def same4(dev, it):
    """Round 6: same-row tap reuse forced on (render_same=1) for the square config 4 (the camera path's
    zoom makes some rows stay on their texel row): 125 and 1 views, gathers counted by the census build."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(0)
    view = torch.rand((H, W, P, 4), generator=g, device=dev)
    packed = _lib.pack_planes(view)
    del view
    for V in (125, 1):
        homs = _host.render_homographies(configs.f32(c["poses"][:V]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]] * V), V).to(dev)
        out = torch.empty((V, H, W, 3), device=dev)
        vs = [("auto", {}), ("same", {"render_same": 1})]
        frames, counts = [], []
        for label, opts in vs:
            with _lib.debug(**opts):
                census = torch.zeros(1, dtype=torch.int64, device=dev)
                _lib._call("mpiv_render_packed_census", packed, H, W, P, homs, V, out, census, _lib._stream(dev))
                torch.cuda.synchronize()
                frames.append(out.clone())
                counts.append(int(census.item()))
        print(json.dumps({"exp": f"same4 census, c4 {V} views", "gathers": counts,
                          "per_sample": [round(n / (V * H * W * P / 64), 4) for n in counts],
                          "same": bool(torch.equal(frames[0].view(torch.int32), frames[1].view(torch.int32)))}),
              flush=True)
        del frames
        fn = lambda: _lib._call("mpiv_render_packed", packed, H, W, P, homs, V, out, _lib._stream(dev))  # noqa: E731
        run(f"c4 packed render, {V} views", vs, fn, V * (P * H * W * 16 + H * W * 12), max(3, it // (1 + V // 8)))
        del out


def same1(dev, it):
    """Round 6: config 2 at one view per launch (288 tiles of 64 x 32: the one-row kernel by default)
    against the same-row reuse kernel forced (render_vshare=4), and the u8 / ct variants' inputs."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(0)
    view = torch.rand((H, W, P, 4), generator=g, device=dev)
    packed = _lib.pack_planes(view)
    del view
    for k in (0, 5, 20):
        homs = _host.render_homographies(configs.f32(c["poses"][k:k + 1]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]]), 1).to(dev)
        out = torch.empty((1, H, W, 3), device=dev)
        fn = lambda: _lib._call("mpiv_render_packed", packed, H, W, P, homs, 1, out, _lib._stream(dev))  # noqa: E731
        vs = [("one_row", {}), ("r6d3_same", {"render_vshare": 4}), ("r4d4_same", {"render_vshare": 11}),
              ("r4d4", {"render_vshare": 11, "render_same": -1})]
        run(f"c2 packed render, 1 view, pose {k}", vs, fn, P * H * W * 16 + H * W * 12, it)


def libs(dev, it):
    """Default routes of the bench legs, for A/B across library builds (MPIV_LIB): config 4 packed at
    1 and 125 views, u8 single view, in-place single view, the fused net-output view, config 5's shard."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    mpi, homs1, _, _, _ = c4_mpi(dev)
    packed = _lib.pack_planes(mpi[0])
    out1 = torch.empty((1, H, W, 3), device=dev)
    per_view = P * H * W * 16 + H * W * 12
    run("c4 packed 1 view", DEF, lambda: _lib.render_packed(packed, homs1, out1), per_view, it)
    run("c4 in-place 1 view", DEF, lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs1, out1,
                                                      _lib._stream(dev)), per_view, it)
    homs = _host.render_homographies(configs.f32(c["poses"][:125]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]] * 125), 125).to(dev)
    out = torch.empty((125, H, W, 3), device=dev)
    run("c4 packed 125 views", DEF, lambda: _lib.render_packed(packed, homs, out), 125 * per_view, 3)
    del out, mpi
    pk8 = _lib.synth_mpi_packed_u8(c["seed"], H, W, 0, P, dev)
    run("u8 c4 1 view", DEF, lambda: _lib._call("mpiv_render_packed_u8", pk8, H, W, P, homs1, 1, out1,
                                                _lib._stream(dev)), P * H * W * 4 + H * W * 12, it)
    del pk8, packed
    c2 = configs.config2()
    H, W, P = c2["H"], c2["W"], c2["P"]
    g = torch.Generator(device=dev).manual_seed(c2["seed"])
    pred = torch.rand((1, 2 * P + 3, H, W), generator=g, device=dev) * 2 - 1
    fg = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    h2 = _host.render_homographies(configs.f32(c2["poses"][5:6]), configs.f32(c2["depths"]), configs.f32([c2["K"]]),
                                   1).to(dev)
    o2 = torch.empty((1, H, W, 3), device=dev)
    run("netout c2 1 view", DEF, lambda: _lib._call("mpiv_render_net_output", pred, _lib._strides(pred), fg,
                                                    _lib._strides(fg), 1, H, W, P, h2, o2, _lib._stream(dev)),
        H * W * ((2 * P + 3) * 4 + 24), it)
    packed2 = _lib.pack_planes(torch.rand((H, W, P, 4), generator=g, device=dev))
    V2 = len(c2["poses"])
    h64 = _host.render_homographies(configs.f32(c2["poses"]), configs.f32(c2["depths"]), configs.f32([c2["K"]] * V2),
                                    V2).to(dev)
    o64 = torch.empty((V2, H, W, 3), device=dev)
    run("c2 packed 64 views", DEF, lambda: _lib.render_packed(packed2, h64, o64), V2 * (P * H * W * 16 + H * W * 12), it)
    del packed2, o64
    c5c = configs.config5()
    H, W, P = c5c["H"], c5c["W"], c5c["P"]
    PL = P // 8
    pk = torch.zeros(_lib.packed_shape(H, W, PL), device=dev)
    pk[:, 2:2 + H, 2:2 + W].uniform_(generator=g)
    h5 = _host.render_homographies(configs.f32(c5c["poses"]), configs.f32(c5c["depths"]), configs.f32([c5c["K"]]),
                                   1)[:, :PL].contiguous().to(dev)
    ct = torch.empty((1, H, W, 4), device=dev)
    run("c5 shard", DEF, lambda: _lib.render_packed_ct(pk, h5, back=True, out=ct), PL * H * W * 16 + H * W * 16, it)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="chunk,train,bwd")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in a.only.split(","):
        globals()[name](dev, a.iters)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

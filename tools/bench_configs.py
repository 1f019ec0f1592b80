#!/usr/bin/env python3
"""Per-config GPU timings for every BASELINE.json config (bench.py covers the
headline config 4).  One JSON line per measurement: kernel time from HIP events
on the launching stream (median of --iters after --warmup), throughput and the
achieved fraction of the 8 TB/s HBM roofline on ALGORITHMIC bytes.

    python tools/bench_configs.py [--iters 20] [--only c1,c2,c3,c4,c5,bwd,net]
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

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

PEAK = 8000.0


def timed(fn, iters, warmup):
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


def report(name, ms, ms_min, alg_bytes, mpix=None, extra=None):
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    r = {"config": name, "ms_median": round(ms, 4), "ms_min": round(ms_min, 4), "alg_GB": round(alg_bytes / 1e9, 4),
         "achieved_GBs": round(gbs, 1), "roofline_frac": round(gbs / PEAK, 4)}
    if mpix is not None:
        r["Mpix_per_s"] = round(mpix / (ms * 1e-3), 1)
    if extra:
        r.update(extra)
    print(json.dumps(r), flush=True)


def gen_mpi(H, W, P, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    m = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    m[..., :3].mul_(2).sub_(1)
    m[:, :, :, 0, 3] = 1.0
    return m


def c1(dev, it, wu):
    c = configs.config1_camera()
    H, W, P = c["H"], c["W"], c["P"]
    mpi = gen_mpi(H, W, P, 0, dev)
    pose = configs.f32(c["poses"][:1]).to(dev)
    K = configs.f32([c["K"]]).to(dev)
    d = configs.f32(c["depths"]).to(dev)
    ms, mn = timed(lambda: mv.mpi_render_view_torch(mpi, pose, d, K), it, wu)
    report("c1 test-MPI 640x400x10, 1 pose, mpi_render_view_torch end-to-end (host H + native kernel)", ms, mn,
           P * H * W * 16 + H * W * 12, H * W / 1e6)
    homs = _host.render_homographies(pose, d, K, 1).to(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    ms, mn = timed(lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out,
                                      _lib._stream(dev)), it, wu)
    report("c1 native kernel only", ms, mn, P * H * W * 16 + H * W * 12, H * W / 1e6)


def c2(dev, it, wu):
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    V = len(c["poses"])
    mpi = gen_mpi(H, W, P, 0, dev)
    homs = _host.render_homographies(configs.f32(c["poses"]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]] * V), V).to(dev)
    packed = _lib.pack_planes(mpi[0])
    out = torch.empty((V, H, W, 3), device=dev)
    per_view = P * H * W * 16 + H * W * 12
    for label, opts in (("default routing", {}), ("direct gathers", {"render_tile": -1}),
                        ("multi-view LDS kernel", {"render_mv": 1}), ("rows x8 per lane", {"render_tile": 8}),
                        ("rows x8, vertical tap reuse", {"render_tile": 8, "render_vshare": 1}),
                        ("rows x8, vertical reuse, 4 rows in flight", {"render_vshare": 3}),
                        ("rows x9, vertical reuse, 3 rows in flight", {"render_vshare": 5}),
                        ("rows x6, vertical reuse, 3 rows in flight", {"render_vshare": 4}),
                        ("rows x9, vertical reuse, 3 rows in flight (again)", {"render_vshare": 5})):
        with _lib.debug(**opts):
            ms, mn = timed(lambda: _lib.render_packed(packed, homs, out), it, wu)
        report(f"c2 1024x576x32, {V} views, packed, {label}", ms, mn, V * per_view, V * H * W / 1e6)
    for V1 in (1, 8):
        h1 = homs[:V1].contiguous()
        o1 = out[:V1]
        for label, opts in (("default routing", {}), ("direct gathers", {"render_tile": -1}),
                            ("rows x8, vertical tap reuse", {"render_tile": 8, "render_vshare": 1}),
                            ("rows x8, vertical reuse, 4 rows in flight", {"render_vshare": 3}),
                            ("rows x4, vertical reuse, 4 rows in flight", {"render_vshare": 11})):
            with _lib.debug(**opts):
                ms, mn = timed(lambda: _lib.render_packed(packed, h1, o1), it, wu)
            report(f"c2 1024x576x32, {V1} views, packed, {label}", ms, mn, V1 * per_view, V1 * H * W / 1e6)
    ms, mn = timed(lambda: _lib.pack_planes(mpi[0]), it, wu)
    report("c2 pack (one-time per MPI)", ms, mn, 2 * P * H * W * 16)
    mpi5 = mpi.expand(V, H, W, P, 4)
    ms, mn = timed(lambda: _lib._call("mpiv_render", mpi5, _lib._strides(mpi5), V, H, W, P, homs, out,
                                      _lib._stream(dev)), max(3, it // 4), 1)
    report(f"c2 native kernel, {V} views (no pack)", ms, mn, V * per_view, V * H * W / 1e6)


def c3(dev, it, wu):
    c = configs.config3()
    S, H, W, D = c["S"], c["H"], c["W"], c["D"]
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.rand((S, H, W, 3), generator=g, device=dev)
    K = configs.f32([c["K"]] * S)
    ki, proj = _host.psv_matrices(K, K, configs.f32(c["poses"]))
    ki, proj = ki.to(dev), proj.to(dev)
    d = configs.f32(c["depths"]).to(dev)
    out = torch.empty((S, H, W, D * 3), device=dev)
    fn = lambda: _lib._call("mpiv_plane_sweep", img, _lib._strides(img), S, H, W, 3, ki, proj, d, D, H, W, out,  # noqa: E731
                            _lib._stream(dev))
    alg = S * H * W * 12 + S * D * H * W * 12
    img4 = _lib.pad_texels(img)  # [S, H+4, W+4, 4]
    pad = lambda: _lib.pad_texels(img, out=img4)  # noqa: E731
    sweep = lambda: _lib._call("mpiv_plane_sweep_padded", img4, S, H, W, 3, ki, proj, d, D, H, W, out,  # noqa: E731
                               _lib._stream(dev))
    pad()
    ms, mn = timed(lambda: out.fill_(1.0), it, wu)
    report(f"c3 write-bandwidth reference: torch fill_ of the {S}x{H}x{W}x{D * 3} volume", ms, mn,
           S * D * H * W * 12)
    for label, opts in (("pixel-per-lane LDS kernel (warm-up)", {"sweep_dlane": 0}),
                        ("depth-per-lane LDS kernel (default)", {}), ("pixel-per-lane LDS kernel", {"sweep_dlane": 0}),
                        ("depth-per-lane LDS kernel (default), again", {}),
                        ("pixel-per-lane LDS kernel, again", {"sweep_dlane": 0}), ("tile kernel", {"sweep_tile": 1}),
                        ("grouped kernel, store mode 1", {"sweep_store": 1}),
                        ("grouped kernel, store mode 2", {"sweep_store": 2})):
        with _lib.debug(**opts):
            ms, mn = timed(sweep, it, wu)
        report(f"c3 PSV {S}x{H}x{W}x3 -> {D} planes, {label}", ms, mn, alg,
               extra={"Mplanepix_per_s": round(S * D * H * W / 1e6 / (ms * 1e-3), 1)})
    # the notebook's dataset PSV: 10 planes (inv_depths(1, 100, 10), ipynb cell 8 L73)
    d10 = configs.f32(configs.inv_depths(1, 100, 10)).to(dev)
    out10 = torch.empty((S, H, W, 10 * 3), device=dev)
    sweep10 = lambda: _lib._call("mpiv_plane_sweep_padded", img4, S, H, W, 3, ki, proj, d10, 10, H, W, out10,  # noqa: E731
                                 _lib._stream(dev))
    alg10 = S * H * W * 12 + S * 10 * H * W * 12
    for label, opts in (("depth-per-lane (default)", {}), ("pixel-per-lane", {"sweep_dlane": 0})):
        with _lib.debug(**opts):
            ms, mn = timed(sweep10, it, wu)
        report(f"c3 sources, 10 planes (notebook dataset PSV), {label}", ms, mn, alg10)
    ms, mn = timed(fn, it, wu)
    report(f"c3 PSV {S}x{H}x{W}x3 -> {D} planes, mpiv_plane_sweep: depth-per-lane on the source in place "
           "(the plane_sweep_torch path)", ms, mn, alg,
           extra={"Mplanepix_per_s": round(S * D * H * W / 1e6 / (ms * 1e-3), 1)})
    with _lib.debug(sweep_dlane=0):
        ms, mn = timed(fn, it, wu)
    report(f"c3 PSV {S}x{H}x{W}x3 -> {D} planes, mpiv_plane_sweep with sweep_dlane=0: generic strided kernel",
           ms, mn, alg)
    ms, mn = timed(lambda: (pad(), sweep()), it, wu)
    report("c3 PSV pad + padded depth-per-lane kernel", ms, mn, alg,
           extra={"Mplanepix_per_s": round(S * D * H * W / 1e6 / (ms * 1e-3), 1)})


def c4(dev, it, wu):
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    mpi = gen_mpi(H, W, P, 0, dev)
    packed = _lib.pack_planes(mpi[0])
    per_view = P * H * W * 16 + H * W * 12
    for V in (1, 8, 125):
        homs = _host.render_homographies(configs.f32(c["poses"][:V]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]] * V), V).to(dev)
        out = torch.empty((V, H, W, 3), device=dev)
        n_it = it if V < 125 else max(3, it // 4)
        for label, opts in (("default routing", {}), ("direct gathers", {"render_tile": -1}),
                            ("multi-view LDS kernel", {"render_mv": 1}),
                            ("LDS-DMA ring 8w 64x8/2", {"render_ring": 4}), ("rows x8 per lane", {"render_tile": 8}),
                            ("rows x8, vertical tap reuse", {"render_tile": 8, "render_vshare": 1}),
                            ("rows x8, vertical reuse, 4 rows in flight", {"render_vshare": 3}),
                            ("rows x6, vertical reuse, 3 rows in flight", {"render_vshare": 4}),
                            ("rows x9, vertical reuse, 3 rows in flight", {"render_vshare": 5}),
                            ("rows x4, vertical reuse, 4 rows in flight", {"render_vshare": 11}),
                            ("rows x4, vertical reuse, 4 rows in flight (again)", {"render_vshare": 11}),
                            ("rows x8, vertical reuse, 4 rows in flight (again)", {"render_vshare": 3}),
                            ("rows x6, vertical reuse, 3 rows in flight (again)", {"render_vshare": 4}),
                            ("rows x8, vertical tap reuse (again)", {"render_tile": 8, "render_vshare": 1}),
                            ("rows x16 per lane", {"render_tile": 16})):
            if V == 125 and ("ring" in label or "LDS kernel" in label):
                continue
            with _lib.debug(**opts):
                ms, mn = timed(lambda: _lib.render_packed(packed, homs, out), n_it, 1)
            report(f"c4 1024^2x128 packed, {label}, {V} views/launch", ms, mn, V * per_view, V * H * W / 1e6)
        ms, mn = timed(lambda: _lib._call("mpiv_render_packed_lds", packed, H, W, P, homs, V, out,
                                          _lib._stream(dev)), n_it, 1)
        report(f"c4 1024^2x128 packed, single-view LDS variant, {V} views/launch", ms, mn, V * per_view,
               V * H * W / 1e6)
    homs = _host.render_homographies(configs.f32(c["poses"][:1]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1).to(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    for label, opts in (("chunked CH=8 (default)", {}), ("chunked CH=4", {"render_chunk": 4}),
                        ("one pixel per lane", {"render_chunk": -1})):
        with _lib.debug(**opts):
            ms, mn = timed(lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out,
                                              _lib._stream(dev)), it, wu)
        report(f"c4 in-place kernel (reference layout), {label}, 1 view", ms, mn, per_view, H * W / 1e6)
    pose = configs.f32(c["poses"][:1]).to(dev)
    K = configs.f32([c["K"]]).to(dev)
    d = configs.f32(c["depths"]).to(dev)
    for policy in ("auto", "pack"):
        _lib.RENDER_POLICY = policy
        ms, mn = timed(lambda: mv.mpi_render_view_torch(mpi, pose, d, K), it, wu)
        report(f"c4 mpi_render_view_torch end-to-end, 1 view, policy={policy}", ms, mn, per_view, H * W / 1e6)
    _lib.RENDER_POLICY = "auto"


def c4n(dev, it, wu):
    """Config 4 through the in-place (reference layout) kernels only: chunked variants
    (render_chunk = CH, +100 = two composite phases per chunk) and the drop-in."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    mpi = gen_mpi(H, W, P, 0, dev)
    per_view = P * H * W * 16 + H * W * 12
    homs = _host.render_homographies(configs.f32(c["poses"][:1]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1).to(dev)
    out = torch.empty((1, H, W, 3), device=dev)
    for opt in (0, 8, 108, 4, 104):
        with _lib.debug(render_chunk=opt):
            ms, mn = timed(lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out,
                                              _lib._stream(dev)), it, wu)
        report(f"c4 in-place kernel, render_chunk={opt}, 1 view", ms, mn, per_view, H * W / 1e6)
    pose = configs.f32(c["poses"][:1]).to(dev)
    K = configs.f32([c["K"]]).to(dev)
    d = configs.f32(c["depths"]).to(dev)
    ms, mn = timed(lambda: mv.mpi_render_view_torch(mpi, pose, d, K), it, wu)
    report("c4 mpi_render_view_torch end-to-end, 1 view (default routing)", ms, mn, per_view, H * W / 1e6)


def u8(dev, it, wu):
    """8-bit RGBA MPIs (render_u8.hip): config 4 at 1 / 8 / 125 views per launch and the
    config-5 plane shard, u8 texels (4 B) vs the float path (16 B).  Bytes are the u8
    algorithmic bytes P*H*W*4 + H*W*12 per view (shard: (P/G)*H*W*4 + H*W*16)."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    packed = _lib.synth_mpi_packed_u8(0, H, W, 0, P, dev)
    per_view = P * H * W * 4 + H * W * 12
    for V in (1, 8, 125):
        homs = _host.render_homographies(configs.f32(c["poses"][:V]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]] * V), V).to(dev)
        out = torch.empty((V, H, W, 3), device=dev)
        for label, opts in (("default routing", {}), ("2 rows per lane", {"render_tile": 2}),
                            ("8 rows per lane", {"render_tile": 8}),
                            ("4 rows, vertical tap reuse", {"render_tile": 4, "render_vshare": 1}),
                            ("8 rows, vertical tap reuse", {"render_tile": 8, "render_vshare": 1})):
            with _lib.debug(**opts):
                ms, mn = timed(lambda: _lib.render_packed_u8(packed, homs, out), it if V < 125 else 3, 1)
            report(f"u8 c4 1024^2x128 u8 texels, {label}, {V} views/launch", ms, mn, V * per_view, V * H * W / 1e6)
    del packed
    c5c = configs.config5()
    H, W, P = c5c["H"], c5c["W"], c5c["P"]
    PL = P // 8
    packed = _lib.synth_mpi_packed_u8(0, H, W, 0, PL, dev)
    homs = _host.render_homographies(configs.f32(c5c["poses"]), configs.f32(c5c["depths"]),
                                     configs.f32([c5c["K"]]), 1)[:, :PL].contiguous().to(dev)
    ct = torch.empty((1, H, W, 4), device=dev)
    for label, opts in (("default routing", {}), ("8 rows per lane", {"render_tile": 8}),
                        ("4 rows, vertical tap reuse", {"render_tile": 4, "render_vshare": 1}),
                        ("8 rows, vertical tap reuse", {"render_tile": 8, "render_vshare": 1})):
        with _lib.debug(**opts):
            ms, mn = timed(lambda: _lib.render_packed_u8_ct(packed, homs, back=True, out=ct), it, wu)
        report(f"u8 c5 plane shard: {PL} of {P} planes, 4096x2160 u8 texels, (C,T), {label}", ms, mn,
               PL * H * W * 4 + H * W * 16, H * W / 1e6)
    del packed
    c2c = configs.config2()  # a stretched MPI (x step W/(H-1) = 1.78), small and large launches
    H, W, P = c2c["H"], c2c["W"], c2c["P"]
    packed = _lib.synth_mpi_packed_u8(0, H, W, 0, P, dev)
    per_view = P * H * W * 4 + H * W * 12
    V2 = len(c2c["poses"])
    homs_all = _host.render_homographies(configs.f32(c2c["poses"]), configs.f32(c2c["depths"]),
                                         configs.f32([c2c["K"]] * V2), V2).to(dev)
    for V in (1, 8, V2):
        homs = homs_all[:V].contiguous()
        out = torch.empty((V, H, W, 3), device=dev)
        for label, opts in (("default routing", {}), ("2 rows per lane", {"render_tile": 2}),
                            ("4 rows, vertical tap reuse", {"render_tile": 4, "render_vshare": 1}),
                            ("2 rows per lane (again)", {"render_tile": 2})):
            with _lib.debug(**opts):
                ms, mn = timed(lambda: _lib.render_packed_u8(packed, homs, out), it, wu)
            report(f"u8 c2 {W}x{H}x{P} u8 texels, {label}, {V} views/launch", ms, mn, V * per_view, V * H * W / 1e6)


def c5(dev, it, wu):
    """Per-GPU share of the 8-way plane-sharded 4096x2160x256 render + the combine."""
    c = configs.config5()
    H, W, P = c["H"], c["W"], c["P"]
    G = 8
    PL = P // G
    g = torch.Generator(device=dev).manual_seed(0)
    packed = torch.zeros(_lib.packed_shape(H, W, PL), device=dev)
    packed[:, 2:2 + H, 2:2 + W].uniform_(generator=g)
    homs = _host.render_homographies(configs.f32(c["poses"]), configs.f32(c["depths"]), configs.f32([c["K"]]), 1)
    homs_local = homs[:, :PL].contiguous().to(dev)
    ct = torch.empty((1, H, W, 4), device=dev)
    for label, opts in (("default routing", {}), ("direct gathers", {"render_tile": -1}),
                        ("LDS-DMA ring 8w 64x8/2", {"render_ring": 4}), ("rows x8 per lane", {"render_tile": 8}),
                            ("rows x8, vertical tap reuse", {"render_tile": 8, "render_vshare": 1}),
                            ("rows x8, vertical reuse, 4 rows in flight", {"render_vshare": 3}),
                            ("rows x9, vertical reuse, 3 rows in flight", {"render_vshare": 5}),
                            ("rows x4, vertical reuse, 4 rows in flight", {"render_vshare": 11}),
                            ("rows x8, vertical reuse, 4 rows in flight (again)", {"render_vshare": 3}),
                            ("rows x16 per lane", {"render_tile": 16})):
        with _lib.debug(**opts):
            ms, mn = timed(lambda: _lib.render_packed_ct(packed, homs_local, back=True, out=ct), it, wu)
        report(f"c5 plane shard: {PL} of {P} planes, 4096x2160 partial (C,T), {label}", ms, mn,
               PL * H * W * 16 + H * W * 16, H * W / 1e6)
    bh = H // G
    parts = torch.rand((G, 1, bh, W, 4), device=dev)
    ms, mn = timed(lambda: _lib.combine_ct(parts), it, wu)
    report(f"c5 ordered combine of {G} band partials ({bh}x{W})", ms, mn, G * bh * W * 16 + bh * W * 12)


def bwd(dev, it, wu):
    """Render backward (d render / d rgba_layers, bit-exact adjoint) per view at the
    config-2 and config-4 sizes; bytes = the MPI read by the forward recompute + its
    gradient written (P*H*W*32) -- the workspace traffic is reported, not counted."""
    for name, c in (("c2", configs.config2()), ("c4", configs.config4())):
        H, W, P = c["H"], c["W"], c["P"]
        mpi = gen_mpi(H, W, P, 0, dev)
        homs = _host.render_homographies(configs.f32(c["poses"][:1]), configs.f32(c["depths"]),
                                         configs.f32([c["K"]]), 1)
        dout = torch.rand((1, H, W, 3), device=dev) * 2 - 1
        ms, mn = timed(lambda: _lib.render_backward(mpi, homs, dout), max(3, it // 4), 1)
        ws = _lib.load().mpiv_render_backward_workspace_size(H, W, P)
        report(f"{name} render backward {W}x{H}x{P}, 1 view, no forward checkpoints (chain 2 passes + gather)", ms,
               mn, P * H * W * 32, H * W / 1e6, extra={"workspace_GB": round(ws / 1e9, 3)})
        hd = homs.to(dev)
        ms, mn = timed(lambda: _lib.render_train(mpi, hd), max(3, it // 4), 1)
        report(f"{name} training forward {W}x{H}x{P}, 1 view (frame + composite checkpoints)", ms, mn,
               P * H * W * 16 + H * W * 12 + (P + 7) // 8 * H * W * 16, H * W / 1e6)
        _, ck = _lib.render_train(mpi, hd)
        ms, mn = timed(lambda: _lib.render_backward(mpi, hd, dout, ckpt=ck), max(3, it // 4), 1)
        report(f"{name} render backward {W}x{H}x{P}, 1 view, forward checkpoints (chain 1 pass + gather)", ms, mn,
               P * H * W * 32, H * W / 1e6, extra={"workspace_GB": round(ws / 1e9, 3)})


def _notebook_assembly(mpi_pred, ref_img, P):
    """The notebook's mpi_from_net_output op sequence (ipynb cell 10 L79-111: P-step
    torch.cat loop) on torch's GPU ops -- the reference path on this GPU, for comparison."""
    B, _, H, W = mpi_pred.shape
    p = mpi_pred.permute(0, 2, 3, 1)
    bw = (p[..., :P] + 1.) / 2.
    al = (p[..., P:2 * P] + 1.) / 2.
    bg = p[..., -3:]
    layers = None
    for i in range(P):
        w = bw[..., i:i + 1]
        cur = torch.cat([w * ref_img + (1 - w) * bg, al[..., i:i + 1]], dim=3)
        layers = cur if layers is None else torch.cat([layers, cur], dim=3)
    return layers.reshape(B, H, W, P, 4)


def net(dev, it, wu):
    """MPI assembly from the network output at the config-2 size (Stereo-Mag 1024x576x32,
    one view): bytes = prediction (2P+3)*4 + reference image 12 read + the MPI written
    (P*16 per pixel); packed layout writes the padded planes."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(3)
    pred = torch.rand((1, 2 * P + 3, H, W), generator=g, device=dev) * 2 - 1
    ref = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    alg = H * W * ((2 * P + 3) * 4 + 12 + P * 16)
    ms, mn = timed(lambda: _lib.assemble_mpi(pred, ref, P), it, wu)
    report(f"net assemble {W}x{H}x{P} -> [1,H,W,P,4] (HIP)", ms, mn, alg, H * W / 1e6)
    packed = torch.empty(_lib.packed_shape(H, W, P), device=dev)
    ms, mn = timed(lambda: _lib.assemble_mpi_packed(pred, ref, P, 0, out=packed), it, wu)
    report(f"net assemble {W}x{H}x{P} -> packed planes (HIP)", ms, mn,
           H * W * ((2 * P + 3) * 4 + 12) + (H + 4) * (W + 4) * P * 16, H * W / 1e6)
    ms, mn = timed(lambda: _notebook_assembly(pred, ref, P), max(3, it // 4), 1)
    report(f"net assemble {W}x{H}x{P}: the notebook's torch.cat loop on torch GPU ops", ms, mn, alg, H * W / 1e6)
    drgba = torch.rand((1, H, W, P, 4), generator=g, device=dev) * 2 - 1
    ms, mn = timed(lambda: _lib.assemble_mpi_backward(drgba, pred, ref, P), it, wu)
    report(f"net assemble backward {W}x{H}x{P} (HIP)", ms, mn, H * W * (P * 16 + (2 * P + 3) * 8 + 12), H * W / 1e6)
    K = configs.f32([c["K"]]).to(dev)
    pose = configs.f32(c["poses"][:1]).to(dev)
    planes = configs.f32(c["depths"]).to(dev)
    ms, mn = timed(lambda: mv.mpi_render_net_output_torch(pred, ref, pose, planes, K), it, wu)
    report(f"net output -> rendered view {W}x{H}x{P}, one kernel (drop-in end to end)", ms, mn,
           H * W * ((2 * P + 3) * 4 + 12 + 12), H * W / 1e6)
    homs = _host.render_homographies(pose, planes, K, 1).to(dev)
    ms, mn = timed(lambda: _lib.render_net_output(pred, ref, P, homs), it, wu)
    report(f"net output -> rendered view {W}x{H}x{P}, one kernel (render_netout_kernel only)", ms, mn,
           H * W * ((2 * P + 3) * 4 + 12 + 12), H * W / 1e6)
    pk = torch.empty(_lib.packed_shape(H, W, P), device=dev)
    o1 = torch.empty((1, H, W, 3), device=dev)
    ms, mn = timed(lambda: (_lib.assemble_mpi_packed(pred, ref, P, 0, out=pk), _lib.render_packed(pk, homs, out=o1)),
                   it, wu)
    report(f"net output -> rendered view {W}x{H}x{P}, two launches (assemble to packed + render)", ms, mn,
           alg + P * H * W * 16 + H * W * 12, H * W / 1e6)
    dep = {"mpi_planes": torch.zeros((1, P), device=dev), "ref_img": ref}
    ms, mn = timed(lambda: mv.mpi_render_view_torch(mv.mpi_from_net_output(pred, dep), pose, planes, K), it, wu)
    report(f"net output -> rendered view {W}x{H}x{P}, two-step drop-ins", ms, mn,
           alg + P * H * W * 16 + H * W * 12, H * W / 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", default="c1,c2,c3,c4,c5,u8,bwd,net")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in a.only.split(","):
        globals()[name](dev, a.iters, a.warmup)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""ctypes wrapper around oracle/libmpiv_oracle.so -- TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
as the checker; the product package (mpi_vision_amd) never imports it.
Pinned against the reference's outputs in tests/golden/ (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libmpiv_oracle.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i64 = ctypes.POINTER(ctypes.c_int64)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_render.argtypes = [_f, _i64] + [ctypes.c_int] * 4 + [_f, _f, ctypes.c_int]
        L.oracle_render_ct.argtypes = [_f, _i64] + [ctypes.c_int] * 7 + [_f, _f, ctypes.c_int]
        L.oracle_plane_sweep.argtypes = [_f, _i64] + [ctypes.c_int] * 4 + [_f, _f, _f] + \
            [ctypes.c_int] * 3 + [_f, ctypes.c_int]
        L.oracle_grid_sample.argtypes = [_f, _i64] + [ctypes.c_int] * 4 + [_f, ctypes.c_int, ctypes.c_int,
                                                                          _f, _i64, ctypes.c_int]
        L.oracle_over_composite.argtypes = [_f, ctypes.c_int, ctypes.c_int64, _f]
        L.oracle_render_backward.argtypes = [_f, _i64] + [ctypes.c_int] * 4 + [_f, _f, _f, ctypes.c_int,
                                                                             ctypes.c_int]
        L.oracle_inverse_warp.argtypes = [_f, _i64] + [ctypes.c_int] * 4 + [_f, _f, _f, ctypes.c_int, ctypes.c_int,
                                                                          _f, ctypes.c_int]
        L.oracle_synth_mpi.argtypes = [ctypes.c_uint32] + [ctypes.c_int] * 4 + [_f]
        L.oracle_render_synth.argtypes = [ctypes.c_uint32] + [ctypes.c_int] * 7 + [_f, ctypes.c_int, ctypes.c_int,
                                                                                  _f, ctypes.c_int]
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f)


def _strides(a: np.ndarray):
    return (ctypes.c_int64 * a.ndim)(*[s // a.itemsize for s in a.strides])


def _threads(n):
    return int(n if n else os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def render(mpi: np.ndarray, homs: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """mpi [B,H,W,P,4] float32 (any strides, e.g. a broadcast view), homs [B,P,9] -> [B,H,W,3]."""
    assert mpi.dtype == np.float32 and mpi.ndim == 5 and mpi.shape[-1] == 4
    B, H, W, P, _ = mpi.shape
    homs = np.ascontiguousarray(homs, dtype=np.float32).reshape(B, P, 9)
    out = np.empty((B, H, W, 3), np.float32)
    lib().oracle_render(_fp(mpi), _strides(mpi), B, H, W, P, _fp(homs), _fp(out), _threads(nthreads))
    return out


# grid_sampler_2d_backward's chunk width (Vec<float>::size() of the kernel ATen dispatched) on the host that
# produced tests/golden/grad.npz: 8 reproduces every golden bit for bit, 16 does not
GRID_VEC = 8


def render_backward(mpi: np.ndarray, homs: np.ndarray, dout: np.ndarray, vec: int = GRID_VEC,
                    nthreads: int = 0) -> np.ndarray:
    """d(render)/d(mpi) for mpi [B,H,W,P,4] (any strides), homs [B,P,9], dout [B,H,W,3]
    -> [B,H,W,P,4], in the reference autograd's arithmetic order (bit-exact)."""
    assert mpi.dtype == np.float32 and mpi.ndim == 5 and mpi.shape[-1] == 4
    B, H, W, P, _ = mpi.shape
    homs = np.ascontiguousarray(homs, dtype=np.float32).reshape(B, P, 9)
    dout = np.ascontiguousarray(dout, dtype=np.float32).reshape(B, H, W, 3)
    out = np.empty((B, H, W, P, 4), np.float32)
    lib().oracle_render_backward(_fp(mpi), _strides(mpi), B, H, W, P, _fp(homs), _fp(dout), _fp(out), vec,
                                 _threads(nthreads))
    return out


def render_ct(mpi: np.ndarray, homs: np.ndarray, p0: int, p1: int, back: bool, nthreads: int = 0) -> np.ndarray:
    """Plane-range partial (C, T) -> [B,H,W,4] (plane sharding)."""
    assert mpi.dtype == np.float32 and mpi.ndim == 5
    B, H, W, P, _ = mpi.shape
    homs = np.ascontiguousarray(homs, dtype=np.float32).reshape(B, P, 9)
    out = np.empty((B, H, W, 4), np.float32)
    lib().oracle_render_ct(_fp(mpi), _strides(mpi), B, H, W, P, p0, p1, int(back), _fp(homs), _fp(out),
                           _threads(nthreads))
    return out


def combine_ct(parts: np.ndarray) -> np.ndarray:
    """parts [G, ..., 4] ordered back->front -> [..., 3]: (Cf,Tf) o (Cb,Tb) = (Cf + Tf*Cb, Tf*Tb)."""
    acc = parts[-1].astype(np.float32).copy()
    for k in range(parts.shape[0] - 2, -1, -1):
        b = parts[k]
        acc[..., :3] = np.float32(acc[..., 3:4] * b[..., :3] + acc[..., :3])
        acc[..., 3] = acc[..., 3] * b[..., 3]
    return acc[..., :3]


def synth_mpi(seed: int, H: int, W: int, p0: int, p1: int) -> np.ndarray:
    """Planes [p0, p1) of the counter-based synthetic MPI (mpi_vision_amd synth.hip,
    restated) as [H, W, p1-p0, 4] float32."""
    out = np.empty((H, W, p1 - p0, 4), np.float32)
    lib().oracle_synth_mpi(seed & 0xFFFFFFFF, H, W, p0, p1, _fp(out))
    return out


def render_synth(seed: int, H: int, W: int, homs: np.ndarray, y0: int, y1: int, p0: int = 0, p1=None,
                 back: bool = True, ct: bool = False, nthreads: int = 0) -> np.ndarray:
    """Rows [y0, y1) of one view of the synthetic MPI rendered procedurally (no MPI in
    memory): homs [P, 9] (one view); ct=False -> final colour [y1-y0, W, 3] (p0 = 0),
    ct=True -> the (C, T) partial [y1-y0, W, 4] of planes [p0, p1)."""
    homs = np.ascontiguousarray(homs, np.float32).reshape(-1, 9)
    P = homs.shape[0]
    p1 = P if p1 is None else p1
    out = np.empty((y1 - y0, W, 4 if ct else 3), np.float32)
    lib().oracle_render_synth(seed & 0xFFFFFFFF, H, W, P, p0, p1, int(back), int(ct), _fp(homs), y0, y1, _fp(out),
                              _threads(nthreads))
    return out


def plane_sweep(img: np.ndarray, ki: np.ndarray, proj: np.ndarray, depths, tgt_h: int, tgt_w: int,
                nthreads: int = 0) -> np.ndarray:
    """img [B,Hs,Ws,C]; ki [B,9]; proj [B,16]; depths (python floats -> fp32) -> [B,Ht,Wt,D*C]."""
    assert img.dtype == np.float32 and img.ndim == 4
    B, Hs, Ws, C = img.shape
    ki = np.ascontiguousarray(ki, np.float32).reshape(B, 9)
    proj = np.ascontiguousarray(proj, np.float32).reshape(B, 16)
    d = np.asarray(depths, dtype=np.float64).astype(np.float32)
    D = d.shape[0]
    out = np.empty((B, tgt_h, tgt_w, D * C), np.float32)
    lib().oracle_plane_sweep(_fp(img), _strides(img), B, Hs, Ws, C, _fp(ki), _fp(proj), _fp(d), D,
                             tgt_h, tgt_w, _fp(out), _threads(nthreads))
    return out


def inverse_warp(img: np.ndarray, ki: np.ndarray, proj: np.ndarray, depth: np.ndarray, nthreads: int = 0):
    """projective_inverse_warp_torch[2] with a depth map: img [B,Hs,Ws,C], ki [B,9], proj [B,16],
    depth [B,Ht,Wt] -> [B,Ht,Wt,C]."""
    B, Hs, Ws, C = img.shape
    ki = np.ascontiguousarray(ki, np.float32).reshape(B, 9)
    proj = np.ascontiguousarray(proj, np.float32).reshape(B, 16)
    depth = np.ascontiguousarray(depth, np.float32)
    Ht, Wt = depth.shape[1], depth.shape[2]
    out = np.empty((B, Ht, Wt, C), np.float32)
    lib().oracle_inverse_warp(_fp(img), _strides(img), B, Hs, Ws, C, _fp(ki), _fp(proj), _fp(depth), Ht, Wt,
                              _fp(out), _threads(nthreads))
    return out


def grid_sample_nchw(inp: np.ndarray, coords: np.ndarray, out_channels_last: bool,
                     nthreads: int = 0) -> np.ndarray:
    """inp [N,C,Hi,Wi] (any strides), coords [N,Ho,Wo,2] in [0,1] units -> NCHW or NHWC."""
    N, C, Hi, Wi = inp.shape
    coords = np.ascontiguousarray(coords, np.float32)
    _, Ho, Wo, _ = coords.shape
    if out_channels_last:
        out = np.empty((N, Ho, Wo, C), np.float32)
        view = out.transpose(0, 3, 1, 2)
    else:
        out = np.empty((N, C, Ho, Wo), np.float32)
        view = out
    lib().oracle_grid_sample(_fp(inp), _strides(inp), N, C, Hi, Wi, _fp(coords), Ho, Wo, _fp(out),
                             _strides(view), _threads(nthreads))
    return out


def over_composite(layers: np.ndarray) -> np.ndarray:
    """layers [P, ..., 4] -> [..., 3]."""
    layers = np.ascontiguousarray(layers, np.float32)
    P = layers.shape[0]
    n = int(np.prod(layers.shape[1:-1]))
    out = np.empty(layers.shape[1:-1] + (3,), np.float32)
    lib().oracle_over_composite(_fp(layers), P, n, _fp(out))
    return out


# ---------------------------------------------------------------------------
# MPI assembly (the notebook's mpi_from_net_output, ipynb cell 10 L79-111): pure
# elementwise fp32 arithmetic, so numpy float32 ops round exactly like ATen's CPU
# kernels: (x + 1) / 2, w * fg, 1 - w, (1 - w) * bg, the sum -- each rounded once.
# ---------------------------------------------------------------------------

def assemble_mpi(pred: np.ndarray, fg: np.ndarray, P: int) -> np.ndarray:
    """pred [B,2P+3,H,W] + fg [B,H,W,3] -> rgba [B,H,W,P,4]."""
    one, two = np.float32(1), np.float32(2)
    p = np.transpose(pred.astype(np.float32), (0, 2, 3, 1))               # mpi_pred.permute(0, 2, 3, 1)
    w = (p[..., :P] + one) / two                                          # blend weights
    a = (p[..., P:2 * P] + one) / two                                     # alphas
    bg = p[..., -3:]
    rgb = w[..., :, None] * fg[..., None, :] + (one - w)[..., :, None] * bg[..., None, :]
    return np.concatenate([rgb, a[..., None]], axis=-1).astype(np.float32)


def assemble_mpi_backward(drgba: np.ndarray, pred: np.ndarray, fg: np.ndarray, P: int) -> np.ndarray:
    """d pred for d rgba, in autograd's order: per plane dw = (sum_c g*fg + -(sum_c g*bg)) / 2
    (channel sums left to right), dalpha = g_a / 2, and d bg accumulated from the last
    plane to the first (the engine runs the planes' nodes in reverse creation order)."""
    one, two = np.float32(1), np.float32(2)
    p = np.transpose(pred.astype(np.float32), (0, 2, 3, 1))
    w = (p[..., :P] + one) / two
    bg = p[..., -3:]
    g = drgba.astype(np.float32)
    gc = g[..., :3]
    sf = (gc[..., 0] * fg[..., None, 0] + gc[..., 1] * fg[..., None, 1]) + gc[..., 2] * fg[..., None, 2]
    sb = (gc[..., 0] * bg[..., None, 0] + gc[..., 1] * bg[..., None, 1]) + gc[..., 2] * bg[..., None, 2]
    dw = (sf + -sb) / two
    da = g[..., 3] / two
    contrib = gc * (one - w)[..., None]                                   # [B,H,W,P,3]
    dbg = contrib[..., P - 1, :].copy()
    for i in range(P - 2, -1, -1):
        dbg = dbg + contrib[..., i, :]
    d = np.concatenate([dw, da, dbg], axis=-1)                            # [B,H,W,2P+3]
    # autograd sums the SliceBackward gradients of the three slices of mpi_pred (weights, alphas,
    # bg) and the SelectBackward ones of each weight / alpha plane, each zero-filled outside its
    # slice: every entry also receives +0 terms, which turn a -0 into +0 (x + 0 == x otherwise).
    # Visible where d rgba is exactly 0 (texels no output pixel samples: tests/golden/netout_train.npz)
    d = d + np.float32(0)
    return np.ascontiguousarray(np.transpose(d, (0, 3, 1, 2))).astype(np.float32)


def assemble_mpi_backward_fg(drgba: np.ndarray, pred: np.ndarray, P: int) -> np.ndarray:
    """d fg [B,H,W,3] for d rgba: MulBackward of w * fg per plane (g * w), accumulated from
    the last plane to the first like d bg (the same engine order)."""
    one, two = np.float32(1), np.float32(2)
    p = np.transpose(pred.astype(np.float32), (0, 2, 3, 1))
    w = (p[..., :P] + one) / two
    contrib = drgba.astype(np.float32)[..., :3] * w[..., None]           # [B,H,W,P,3]
    dfg = contrib[..., P - 1, :].copy()
    for i in range(P - 2, -1, -1):
        dfg = dfg + contrib[..., i, :]
    return dfg.astype(np.float32)

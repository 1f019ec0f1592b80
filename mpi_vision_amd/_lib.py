"""ctypes binding to libmpiv.so (C ABI: include/mpiv.h) + tensor plumbing.

Every function here launches a hand-written gfx950 kernel on the caller's
current torch stream.  There is no CPU fallback: without a ROCm device or
without the built library these functions raise.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import hashlib
import os
import weakref

import torch
from torch.autograd.function import once_differentiable

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPIV_LIB: another build of the same ABI (kernel A/B tools only, tools/gpu_ab_lib.sh);
# its build id is not checked against the sources in this tree
LIB_PATH = os.environ.get("MPIV_LIB") or os.path.join(_HERE, "libmpiv.so")
# the A/B flavour of the same sources (Makefile: -DMPIV_AB=1): the production kernels plus the
# variants kept for measurement; loaded only while a debug option selects one of them
AB_PATH = os.path.join(_HERE, "libmpiv_ab.so")
_CSRC = os.path.join(_HERE, "csrc")

_c_i64p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p
_int = ctypes.c_int
_i64 = ctypes.c_int64

# name -> argtypes (mirrors include/mpiv.h)
_SIGS = {
    "mpiv_render": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp],
    "mpiv_pack_planes": [_vp, _c_i64p, _int, _int, _int, _vp, _vp],
    "mpiv_render_packed": [_vp, _int, _int, _int, _vp, _int, _vp, _vp],
    "mpiv_render_packed_lds": [_vp, _int, _int, _int, _vp, _int, _vp, _vp],
    "mpiv_render_packed_ct": [_vp, _int, _int, _int, _int, _int, _int, _vp, _int, _vp, _vp],
    "mpiv_render_packed_ct_rows": [_vp, _int, _int, _int, _int, _int, _int, _vp, _int, _int, _int, _vp, _vp],
    "mpiv_combine_ct": [_vp, _int, _i64, _vp, _vp],
    "mpiv_plane_sweep": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _int, _int, _int, _vp, _vp],
    "mpiv_plane_sweep_pose": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _i64, _vp, _vp, _vp, _int, _int, _int,
                              _vp, _vp],
    "mpiv_inverse_warp": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _c_i64p, _int, _int, _vp, _vp],
    "mpiv_grid_sample": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _c_i64p, _int, _int, _vp, _c_i64p, _vp],
    "mpiv_over_composite": [_vp, _int, _i64, _i64, _i64, _vp, _vp],
    "mpiv_transform_points": [_vp, _int, _i64, _vp, _vp, _vp],
    "mpiv_normalize_homogeneous": [_vp, _i64, _int, _vp, _vp],
    "mpiv_pixel2cam": [_vp, _vp, _vp, _int, _i64, _int, _vp, _vp],
    "mpiv_cam2pixel": [_vp, _vp, _int, _i64, _vp, _vp],
    "mpiv_plane_coords": [_vp, _int, _i64, _vp, _int, _int, _vp, _vp],
    "mpiv_selftest_div_const": [_int, _vp, _vp],
    "mpiv_selftest_tickets": [_int, _int, _int, ctypes.c_uint, _vp, _vp, _vp],
    "mpiv_probe_gather": [_vp, ctypes.c_size_t, _int, _int, _vp, _vp],
    "mpiv_mark": [_int, _vp],
    "mpiv_route": [ctypes.c_char_p, _c_i64p, _int, ctypes.c_char_p, _int, _c_i64p],
    "mpiv_pad_texels": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp],
    "mpiv_plane_sweep_padded": [_vp, _int, _int, _int, _int, _vp, _vp, _vp, _int, _int, _int, _vp, _vp],
    "mpiv_preprocess": [_vp, _i64, _vp, _vp],
    "mpiv_deprocess_u8": [_vp, _i64, _vp, _vp],
    "mpiv_render_backward": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp],
    "mpiv_render_backward_watched": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t,
                                     _vp],
    "mpiv_render_backward_status": [_vp, _int, _int, _int, ctypes.POINTER(_int), _vp],
    "mpiv_render_train": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _vp],
    "mpiv_render_packed_census": [_vp, _int, _int, _int, _vp, _int, _vp, _vp, _vp],
    "mpiv_plane_sweep_into": [_vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _int, _int, _int, _vp, _i64, _i64,
                              _vp],
    "mpiv_plane_sweep_padded_into": [_vp, _int, _int, _int, _int, _vp, _vp, _vp, _int, _int, _int, _vp, _i64, _i64,
                                     _vp],
    "mpiv_assemble_mpi": [_vp, _c_i64p, _vp, _c_i64p, _int, _int, _int, _int, _vp, _vp],
    "mpiv_assemble_mpi_packed": [_vp, _c_i64p, _vp, _c_i64p, _int, _int, _int, _int, _vp, _vp],
    "mpiv_assemble_mpi_sampled": [_vp, _c_i64p, _vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp],
    "mpiv_render_homographies": [_vp, _vp, _vp, _vp, _int, _int, _vp],
    "mpiv_render_homographies_device": [_vp, _vp, _vp, _vp, _int, _int, _vp, _vp],
    "mpiv_psv_proj": [_vp, _i64, _vp, _int, _vp],
    "mpiv_psv_proj_device": [_vp, _i64, _vp, _int, _vp, _vp],
    "mpiv_pack_planes_u8": [_vp, _c_i64p, _int, _int, _int, _vp, _vp],
    "mpiv_render_net_output": [_vp, _c_i64p, _vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp],
    "mpiv_render_net_output_train": [_vp, _c_i64p, _vp, _c_i64p, _int, _int, _int, _int, _vp, _vp, _vp, _vp],
    "mpiv_render_packed_u8": [_vp, _int, _int, _int, _vp, _int, _vp, _vp],
    "mpiv_render_packed_u8_ct": [_vp, _int, _int, _int, _int, _int, _int, _vp, _int, _vp, _vp],
    "mpiv_synth_mpi_packed_u8": [ctypes.c_uint32, _int, _int, _int, _int, _vp, _vp],
    "mpiv_unpack_planes_u8": [_vp, _int, _int, _int, _vp, _vp],
    "mpiv_synth_mpi_packed": [ctypes.c_uint32, _int, _int, _int, _int, _vp, _vp],
    "mpiv_assemble_mpi_backward": [_vp, _c_i64p, _vp, _c_i64p, _vp, _c_i64p, _int, _int, _int, _int, _vp, _vp,
                                   _vp],
}
EXPORTS = tuple(_SIGS) + ("mpiv_abi_version", "mpiv_last_error", "mpiv_render_backward_workspace_size",
                          "mpiv_render_backward_abort_flag",
                          "mpiv_render_backward_workspace_size_min", "mpiv_build_id", "mpiv_debug_set")
ABI_VERSION = 14

_lib = None
_lib_ab = None
_override = None  # the A/B library while a debug option selects an A/B kernel

# How mpi_render_view_torch renders a non-broadcast MPI batch: "auto" (the in-place
# chunked kernel when the layout allows it, else pack per view when P >= 8, else read in
# place), "pack", or "native" (mpiv_render, which picks its in-place kernel itself).
RENDER_POLICY = "auto"

_KOOB = 0x7FFFFF00
_CHUNK_LDS = 65536


def chunk_layout_ok(rgba_layers: torch.Tensor) -> bool:
    """True when mpiv_render reads this [B,H,W,P,4] tensor with render_chunk_kernel
    (abi.hip: planes contiguous per pixel, 16-B texels, offsets below the buffer range)."""
    B, H, W, P, C = rgba_layers.shape
    st = rgba_layers.stride()
    if C != 4 or H < 2 or W < 2 or st[4] != 1 or st[3] != 4 or any(s % 4 for s in st[:3]):
        return False
    if rgba_layers.data_ptr() % 16:
        return False
    CH = 4 if P <= 4 else 8
    rec = ((H - 1) * st[1] + (W - 1) * st[2]) * 4 + CH * 16
    return (rec < _KOOB and st[1] // 4 < (1 << 22) and st[2] // 4 < (1 << 22)
            and 4 * 64 * (CH + 1) * 16 + P * 36 <= _CHUNK_LDS)


def source_hash() -> str | None:
    """sha256 (first 16 hex digits) of the library sources listed in csrc/SOURCES, in order
    -- the id the Makefile compiles into libmpiv.so; None when the sources are absent."""
    try:
        with open(os.path.join(_CSRC, "SOURCES")) as f:
            names = f.read().split()
        h = hashlib.sha256()
        for n in names:
            with open(os.path.join(_CSRC, n), "rb") as f:
                h.update(f.read())
        return h.hexdigest()[:16]
    except OSError:
        return None


def _open(path: str, check_id: bool):
    if not os.path.exists(path):
        raise RuntimeError(f"mpi_vision_amd: {path} is missing -- build it first "
                           "(python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(path)
    L.mpiv_build_id.restype = ctypes.c_char_p
    want = source_hash()
    if check_id and want is not None and L.mpiv_build_id().decode() != want:
        raise RuntimeError(f"mpi_vision_amd: {path} was built from other sources (build id "
                           f"{L.mpiv_build_id().decode()}, sources {want}) -- rebuild it "
                           "(python -c 'import __graft_entry__ as g; g.build()')")
    L.mpiv_debug_set.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.mpiv_debug_set.restype = ctypes.c_int
    for name, args in _SIGS.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    L.mpiv_abi_version.restype = ctypes.c_int
    L.mpiv_last_error.restype = ctypes.c_char_p
    L.mpiv_render_backward_workspace_size.argtypes = [_int, _int, _int]
    L.mpiv_render_backward_workspace_size.restype = ctypes.c_size_t
    L.mpiv_render_backward_workspace_size_min.argtypes = [_int, _int, _int]
    L.mpiv_render_backward_workspace_size_min.restype = ctypes.c_size_t
    L.mpiv_render_backward_abort_flag.argtypes = [_int]
    L.mpiv_render_backward_abort_flag.restype = ctypes.c_void_p
    if L.mpiv_abi_version() != ABI_VERSION:
        raise RuntimeError(f"mpi_vision_amd: {path} ABI version mismatch")
    return L


def load_main():
    """The production libmpiv.so (raises if it has not been built, or was built from other
    sources than the ones in this tree)."""
    global _lib
    if _lib is None:
        _lib = _open(LIB_PATH, not os.environ.get("MPIV_LIB"))
    return _lib


def load_ab():
    """libmpiv_ab.so, the A/B flavour (same sources, -DMPIV_AB=1).  Under MPIV_LIB (an A/B
    tool's own build, which compiles every variant) that library serves both roles."""
    global _lib_ab
    if os.environ.get("MPIV_LIB"):
        return load_main()
    if _lib_ab is None:
        _lib_ab = _open(AB_PATH, True)
    return _lib_ab


def load():
    """The library entry points run through: libmpiv.so, or libmpiv_ab.so while a debug
    option selects an A/B kernel (set_debug)."""
    return _override if _override is not None else load_main()


# MPIV_ROCTX=1: every entry-point call is wrapped in a roctx range named after it, so
# `rocprofv3 --marker-trace --kernel-trace` attributes each kernel to its drop-in call
# (tracing only; off by default: no overhead on the launch path).
_ROCTX = None
if os.environ.get("MPIV_ROCTX") == "1":
    try:
        _ROCTX = ctypes.CDLL("/opt/rocm/lib/libroctx64.so")
        _ROCTX.roctxRangePushA.argtypes = [ctypes.c_char_p]
    except OSError:
        _ROCTX = None


# entry points whose only kernels are A/B variants (libmpiv.so refuses them)
_AB_ENTRIES = frozenset({"mpiv_render_packed_lds"})


def _call(name, *args):
    """Call an entry point (an A/B-only one on libmpiv_ab.so).  Tensor arguments are passed as their device pointers and
    stay referenced (alive) for the duration of the call, so temporaries built inline
    cannot be freed and their memory reused by a later argument's allocation."""
    L = load_ab() if name in _AB_ENTRIES else load()
    # (tensor arguments as plain ints: every pointer parameter's argtype is c_void_p)
    cargs = [a.data_ptr() if isinstance(a, torch.Tensor) else a for a in args]
    if _ROCTX is not None:
        _ROCTX.roctxRangePushA(name.encode())
        try:
            rc = getattr(L, name)(*cargs)
        finally:
            _ROCTX.roctxRangePop()
    else:
        rc = getattr(L, name)(*cargs)
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {L.mpiv_last_error().decode()}")


_DEBUG_GEN = 0  # bumped by every set_debug / reset_debug: memos of option-dependent values key on it


def set_debug(**opts):
    """Select non-default kernel variants (tests and A/B tools only; mpiv_debug_set).
    Options that pick a kernel kept for A/B measurement are refused by the production
    library; then the A/B flavour takes them and runs every entry point until reset_debug()."""
    global _override, _DEBUG_GEN
    _DEBUG_GEN += 1
    L = load_main()
    need_ab = False
    for k, v in opts.items():
        if L.mpiv_debug_set(k.encode(), int(v)) != 0:
            msg = L.mpiv_last_error().decode()
            if "libmpiv_ab.so" not in msg:
                L.mpiv_debug_set(b"reset", 0)
                raise ValueError(msg)
            need_ab = True
    if need_ab or (_override is not None and _override is not L):
        # the A/B flavour runs (now, or still from an earlier call): the options go to it too,
        # so successive calls accumulate on whichever library serves the entry points
        if need_ab:
            L.mpiv_debug_set(b"reset", 0)
        A = load_ab()
        for k, v in opts.items():
            if A.mpiv_debug_set(k.encode(), int(v)) != 0:
                msg = A.mpiv_last_error().decode()
                A.mpiv_debug_set(b"reset", 0)
                raise ValueError(msg)
        _override = A


def reset_debug():
    """Every option back to its production default; entry points back on libmpiv.so."""
    global _override, _DEBUG_GEN
    _DEBUG_GEN += 1
    for L in (_lib, _lib_ab):
        if L is not None:
            L.mpiv_debug_set(b"reset", 0)
    _override = None


@contextlib.contextmanager
def debug(**opts):
    """set_debug(**opts) for the duration of the block, e.g.
    ``with _lib.debug(render_mv=1, box_shrink=2): ...``; reset_debug() on exit."""
    try:
        set_debug(**opts)
        yield
    finally:
        reset_debug()


def route(entry: str, *args: int) -> tuple[str, int]:
    """(kernel name, grid work-items) of the kernel an entry point's production dispatch
    would launch for these sizes (mpiv_route: a dry run, nothing launched, no GPU needed)."""
    L = load_main()
    buf = ctypes.create_string_buffer(160)
    grid = ctypes.c_int64(0)
    a = (ctypes.c_int64 * len(args))(*args)
    rc = L.mpiv_route(entry.encode(), a, len(args), buf, len(buf), ctypes.byref(grid))
    if rc != 0:
        raise RuntimeError(f"mpiv_route failed ({rc}): {L.mpiv_last_error().decode()}")
    return buf.value.decode(), grid.value


def _strides(t: torch.Tensor, dims=None):
    st = t.stride() if dims is None else [t.stride(d) for d in dims]
    return (ctypes.c_int64 * len(st))(*st)


def _dev(*tensors):
    """All tensors must be fp32 on one ROCm device; returns that device."""
    dev = None
    for t in tensors:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"expected a torch.Tensor, got {type(t).__name__}")
        if t.device.type != "cuda":
            raise RuntimeError("mpi_vision_amd kernels need ROCm device tensors "
                               f"(got a tensor on {t.device}); there is no CPU path")
        if t.dtype != torch.float32:
            raise RuntimeError(f"expected scalar type Float but found {t.dtype}")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} and {t.device}")
    return dev


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(dev):
    """The current stream of dev as the hipStream_t the entry points take (the raw handle, without
    building a torch Stream object: this runs on every launch)."""
    if _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(dev.index if dev.index is not None else torch.cuda.current_device()))
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _up(x: torch.Tensor, dev) -> torch.Tensor:
    """Upload a small host-computed matrix buffer (contiguous fp32).  A page-locked host
    buffer is copied asynchronously on the current stream (torch's pinned allocator keeps
    it alive until that copy has run)."""
    if x.device.type == "cpu" and x.is_pinned() and x.dtype == torch.float32 and x.is_contiguous():
        return x.to(device=dev, non_blocking=True)
    return x.to(device=dev, dtype=torch.float32).contiguous()


def _p(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _check_out(out: torch.Tensor, shape, dev, what: str) -> torch.Tensor:
    """A caller-supplied output must be a contiguous fp32 tensor of exactly `shape` on
    `dev` (the kernels write it densely; anything else would be out-of-bounds writes)."""
    if (not isinstance(out, torch.Tensor) or tuple(out.shape) != tuple(shape) or not out.is_contiguous()
            or out.dtype != torch.float32 or out.device != dev):
        got = (tuple(out.shape), out.dtype, out.device, out.is_contiguous()) if isinstance(out, torch.Tensor) \
            else type(out).__name__
        raise RuntimeError(f"{what}: out must be a contiguous float32 {tuple(shape)} tensor on {dev}, got {got}")
    return out


# ---------------------------------------------------------------------------
# render
# ---------------------------------------------------------------------------

PAD = 2  # zero-border texels around every packed plane (include/mpiv.h)


def packed_shape(H: int, W: int, P: int):
    return (P, H + 2 * PAD, W + 2 * PAD, 4)


def packed_hw(packed: torch.Tensor):
    """(P, H, W) of a packed MPI [P, H+4, W+4, 4]."""
    if packed.dim() != 4 or packed.shape[-1] != 4 or not packed.is_contiguous():
        raise RuntimeError(f"packed MPI must be a contiguous [P, H+4, W+4, 4] tensor, got {tuple(packed.shape)}")
    return packed.shape[0], packed.shape[1] - 2 * PAD, packed.shape[2] - 2 * PAD


def pack_planes(view: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """One MPI view [H, W, P, 4] (any strides) -> packed plane-major [P, H+4, W+4, 4]
    with a 2-texel zero border (image texel (x, y) of plane p at [p, y+2, x+2])."""
    dev = _dev(view)
    H, W, P, C = view.shape
    if C != 4:
        raise RuntimeError(f"MPI texels must have 4 channels (RGBA), got {C}")
    packed = torch.empty(packed_shape(H, W, P), device=dev, dtype=torch.float32) if out is None else \
        _check_out(out, packed_shape(H, W, P), dev, "pack_planes")
    _call("mpiv_pack_planes", view, _strides(view), H, W, P, packed, _stream(dev))
    return packed


def synth_mpi_packed(seed: int, H: int, W: int, p_begin: int, p_end: int, device,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """Planes [p_begin, p_end) of the counter-based synthetic MPI `seed` (synth.hip),
    generated on `device` straight into the packed layout [p_end-p_begin, H+4, W+4, 4]."""
    dev = torch.device(device)
    shape = packed_shape(H, W, p_end - p_begin)
    packed = torch.empty(shape, device=dev, dtype=torch.float32) if out is None else \
        _check_out(out, shape, dev, "synth_mpi_packed")
    _dev(packed)
    _call("mpiv_synth_mpi_packed", ctypes.c_uint32(seed & 0xFFFFFFFF), H, W, p_begin, p_end, packed, _stream(dev))
    return packed


def pack_planes_u8(view: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """One 8-bit MPI view [H, W, P, 4] uint8 (any strides) -> packed u8 planes
    [P, H+4, W+4] int32 (RGBA bytes of each texel, R lowest) with the zero border."""
    if not isinstance(view, torch.Tensor) or view.dtype != torch.uint8:
        raise RuntimeError("pack_planes_u8 expects a uint8 [H, W, P, 4] tensor")
    if view.device.type != "cuda":
        raise RuntimeError("mpi_vision_amd kernels need ROCm device tensors; there is no CPU path")
    dev = view.device
    H, W, P, C = view.shape
    if C != 4:
        raise RuntimeError(f"MPI texels must have 4 channels (RGBA), got {C}")
    shape = (P, H + 2 * PAD, W + 2 * PAD)
    if out is None:
        packed = torch.empty(shape, device=dev, dtype=torch.int32)
    elif tuple(out.shape) != shape or out.dtype != torch.int32 or not out.is_contiguous() or out.device != dev:
        raise RuntimeError(f"pack_planes_u8: out must be a contiguous int32 {shape} tensor on {dev}")
    else:
        packed = out
    _call("mpiv_pack_planes_u8", view, _strides(view), H, W, P, packed, _stream(dev))
    if out is not None:
        _wrote(packed)
    return packed


def synth_mpi_packed_u8(seed: int, H: int, W: int, p_begin: int, p_end: int, device) -> torch.Tensor:
    """Planes [p_begin, p_end) of the counter-based synthetic u8 MPI `seed`, packed u8."""
    dev = torch.device(device)
    packed = torch.empty((p_end - p_begin, H + 2 * PAD, W + 2 * PAD), device=dev, dtype=torch.int32)
    _call("mpiv_synth_mpi_packed_u8", ctypes.c_uint32(seed & 0xFFFFFFFF), H, W, p_begin, p_end, packed,
          _stream(dev))
    return packed


def _u8_hw(packed: torch.Tensor):
    if packed.dim() != 3 or packed.dtype != torch.int32 or not packed.is_contiguous() or packed.device.type != "cuda":
        raise RuntimeError("packed u8 MPI must be a contiguous int32 [P, H+4, W+4] ROCm tensor")
    return packed.shape[0], packed.shape[1] - 2 * PAD, packed.shape[2] - 2 * PAD


def unpack_planes_u8(packed: torch.Tensor) -> torch.Tensor:
    """packed u8 [P,H+4,W+4] -> the packed float MPI [P,H+4,W+4,4] of u8.float() / 255 (exact)."""
    P, H, W = _u8_hw(packed)
    out = torch.empty(packed_shape(H, W, P), device=packed.device, dtype=torch.float32)
    _call("mpiv_unpack_planes_u8", packed, H, W, P, out, _stream(packed.device))
    return out


# Views per launch from which render_packed_u8 renders an 8-bit MPI through its float copy (the
# float rows kernel at 125 views: 26.6 ms vs 29.8 for the u8 kernel, VALU-bound on the exact
# per-tap conversion; at one view the u8 kernel reads 4x fewer bytes and wins, 0.31 vs 0.38 ms).
U8_FLOAT_MIN_VIEWS = int(os.environ.get("MPIV_U8_FLOAT_MIN_VIEWS", "32"))
_U8_FLOAT: dict = {}


def _wrote(t: torch.Tensor) -> None:
    """A kernel wrote t through ctypes (an out= argument): bump its version counter as a torch
    in-place op would, so memos keyed on it (u8_float_copy) see the new contents."""
    torch.autograd.graph.increment_version(t)


def u8_float_copy(packed: torch.Tensor) -> torch.Tensor:
    """The packed float copy of a packed u8 MPI, memoised per device on the tensor object, its
    storage, version counter and the current stream (a camera path converts its MPI once; an
    in-place edit, a refill through pack_planes_u8(out=) or a new MPI converts again; a copy is
    only read on the stream that made it).  One entry per device: the copy is 4x the u8 MPI
    (2.2 GB at config 4); it is dropped when the u8 MPI is freed, or by clear_u8_float_copies()."""
    dev = packed.device
    key = (id(packed), packed.data_ptr(), packed._version, tuple(packed.shape),
           torch.cuda.current_stream(dev).cuda_stream)
    ent = _U8_FLOAT.get(dev)
    if ent is not None and ent[0] == key and ent[1]() is packed:
        return ent[2]
    _U8_FLOAT.pop(dev, None)  # free the old copy first
    f = unpack_planes_u8(packed)
    _U8_FLOAT[dev] = (key, weakref.ref(packed), f)
    weakref.finalize(packed, _drop_u8_float, dev, key)
    return f


def _drop_u8_float(dev, key) -> None:
    ent = _U8_FLOAT.get(dev)
    if ent is not None and ent[0] == key:
        del _U8_FLOAT[dev]


def clear_u8_float_copies(device=None) -> None:
    """Free the memoised float copies of u8 MPIs (all devices, or `device`'s)."""
    if device is None:
        _U8_FLOAT.clear()
    else:
        _U8_FLOAT.pop(torch.device(device), None)


def render_packed_u8(packed: torch.Tensor, homs: torch.Tensor, out: torch.Tensor | None = None,
                     route_float: bool | None = None) -> torch.Tensor:
    """packed u8 [P,H+4,W+4] + homs [V,P,9] -> [V,H,W,3] fp32, bit-identical to rendering the
    float MPI u8.float() / 255 (render_u8.hip).  Launches of >= U8_FLOAT_MIN_VIEWS views
    (route_float None) render the MPI's exact float copy (u8_float_copy, converted once per MPI)
    with the float kernel instead: the same bits, faster where the texture path binds."""
    P, H, W = _u8_hw(packed)
    if route_float is None:
        route_float = homs.shape[0] >= U8_FLOAT_MIN_VIEWS
    if route_float:
        return render_packed(u8_float_copy(packed), homs, out=out)
    dev = packed.device
    V = homs.shape[0]
    h = _up(homs.reshape(V, P, 9), dev)
    if out is None:
        out = torch.empty((V, H, W, 3), device=dev, dtype=torch.float32)
    else:
        _check_out(out, (V, H, W, 3), dev, "render_packed_u8")
    if V == 0:
        return out
    _call("mpiv_render_packed_u8", packed, H, W, P, h, V, out, _stream(dev))
    return out


def render_packed_u8_ct(packed: torch.Tensor, homs: torch.Tensor, back: bool, p_begin: int = 0,
                        p_end: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Plane-range partial (C, T) [V,H,W,4] of a packed u8 MPI (plane sharding)."""
    P, H, W = _u8_hw(packed)
    dev = packed.device
    p_end = P if p_end is None else p_end
    V = homs.shape[0]
    h = _up(homs.reshape(V, P, 9), dev)
    if out is None:
        out = torch.empty((V, H, W, 4), device=dev, dtype=torch.float32)
    else:
        _check_out(out, (V, H, W, 4), dev, "render_packed_u8_ct")
    _call("mpiv_render_packed_u8_ct", packed, H, W, P, p_begin, p_end, int(back), h, V, out, _stream(dev))
    return out


def unpack_planes(packed: torch.Tensor) -> torch.Tensor:
    """Inverse view of pack_planes: [P, H+4, W+4, 4] -> [H, W, P, 4] (a strided view)."""
    P, H, W = packed_hw(packed)
    return packed[:, PAD:PAD + H, PAD:PAD + W].permute(1, 2, 0, 3)


def render_packed(packed: torch.Tensor, homs: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """packed [P,H+4,W+4,4] + homs [V,P,9] (host or device) -> [V,H,W,3]."""
    dev = _dev(packed)
    P, H, W = packed_hw(packed)
    V = homs.shape[0]
    h = _up(homs.reshape(V, P, 9), dev)
    if out is None:
        out = torch.empty((V, H, W, 3), device=dev, dtype=torch.float32)
    else:
        _check_out(out, (V, H, W, 3), dev, "render_packed")
    if V == 0:
        return out
    _call("mpiv_render_packed", packed, H, W, P, h, V, out, _stream(dev))
    return out


def render_packed_ct(packed: torch.Tensor, homs: torch.Tensor, back: bool, p_begin: int = 0,
                     p_end: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Plane-range partial (C, T) [V,H,W,4] for plane sharding."""
    dev = _dev(packed)
    P, H, W = packed_hw(packed)
    p_end = P if p_end is None else p_end
    V = homs.shape[0]
    h = _up(homs.reshape(V, P, 9), dev)
    if out is None:
        out = torch.empty((V, H, W, 4), device=dev, dtype=torch.float32)
    else:
        _check_out(out, (V, H, W, 4), dev, "render_packed_ct")
    _call("mpiv_render_packed_ct", packed, H, W, P, p_begin, p_end, int(back), h, V, out,
          _stream(dev))
    return out


def render_packed_ct_rows(packed: torch.Tensor, homs: torch.Tensor, back: bool, y_begin: int, y_end: int,
                          out: torch.Tensor, p_begin: int = 0, p_end: int | None = None) -> torch.Tensor:
    """Rows [y_begin, y_end) of render_packed_ct's partial into out [V,H,W,4] (other rows
    untouched): one row band of a plane shard (mpiv_render_packed_ct_rows, same bits)."""
    dev = _dev(packed)
    P, H, W = packed_hw(packed)
    p_end = P if p_end is None else p_end
    V = homs.shape[0]
    h = _up(homs.reshape(V, P, 9), dev)
    _check_out(out, (V, H, W, 4), dev, "render_packed_ct_rows")
    _call("mpiv_render_packed_ct_rows", packed, H, W, P, p_begin, p_end, int(back), h, V, y_begin, y_end, out,
          _stream(dev))
    return out


def combine_ct(parts: torch.Tensor) -> torch.Tensor:
    """parts [G, ..., 4] ordered back->front -> [..., 3]."""
    dev = _dev(parts)
    parts = parts.contiguous()
    G = parts.shape[0]
    n = parts[0].numel() // 4
    out = torch.empty(tuple(parts.shape[1:-1]) + (3,), device=dev, dtype=torch.float32)
    _call("mpiv_combine_ct", parts, G, n, out, _stream(dev))
    return out


def render(rgba_layers: torch.Tensor, homs: torch.Tensor) -> torch.Tensor:
    """rgba_layers [B,H,W,P,4], homs [B,P,9] -> [B,H,W,3].

    A stride-0 (broadcast) batch is packed once into the plane-major layout and
    all B views render from it; otherwise the native-layout kernel reads the
    reference's tensor in place."""
    dev = _dev(rgba_layers)
    if rgba_layers.dim() != 5 or rgba_layers.shape[-1] != 4:
        raise RuntimeError(f"rgba_layers must be [B,H,W,P,4], got {tuple(rgba_layers.shape)}")
    B, H, W, P, _ = rgba_layers.shape
    if homs.shape[0] != B or homs.shape[1] != P:
        raise RuntimeError(f"shape mismatch: MPI batch/planes {B}/{P} vs poses/planes {homs.shape[0]}/{homs.shape[1]}")
    if B > 1 and rgba_layers.stride(0) == 0:
        return render_packed(pack_planes(rgba_layers[0]), homs)
    h = _up(homs, dev)
    out = torch.empty((B, H, W, 3), device=dev, dtype=torch.float32)
    if RENDER_POLICY == "auto" and chunk_layout_ok(rgba_layers):
        # in place, whole 128-B pixel lines per tap instruction (render_chunk.hip): no pack
        _call("mpiv_render", rgba_layers, _strides(rgba_layers), B, H, W, P, h, out, _stream(dev))
        return out
    if RENDER_POLICY == "pack" or (RENDER_POLICY == "auto" and P >= 8 and (H + 4) * (W + 4) * 16 < 0x7FFFFF00):
        # per view: pack its MPI plane-major (one coalesced transpose pass) and render
        # from the packed copy -- the gathers of the in-place layout touch one 128-B
        # line per 16-B texel, which is slower than paying the pack
        packed = torch.empty(packed_shape(H, W, P), device=dev, dtype=torch.float32)
        for b in range(B):
            _call("mpiv_pack_planes", rgba_layers[b], _strides(rgba_layers[b]), H, W, P, packed, _stream(dev))
            _call("mpiv_render_packed", packed, H, W, P, h[b:b + 1], 1, out[b:b + 1], _stream(dev))
        return out
    _call("mpiv_render", rgba_layers, _strides(rgba_layers), B, H, W, P, h, out, _stream(dev))
    return out


def bwd_layout_ok(rgba_layers: torch.Tensor) -> bool:
    """True when mpiv_render_backward reads this [B,H,W,P,4] tensor in place (abi.hip:
    16-B texels with planes contiguous per pixel, one view below the buffer range)."""
    B, H, W, P, C = rgba_layers.shape
    st = rgba_layers.stride()
    if C != 4 or st[4] != 1 or st[3] != 4 or any(s % 4 for s in st[:3]) or st[1] < 0 or st[2] < 0:
        return False
    rec = ((H - 1) * st[1] + (W - 1) * st[2]) * 4 + 8 * 16
    return rgba_layers.data_ptr() % 16 == 0 and rec < _KOOB and st[1] // 4 < (1 << 22) and st[2] // 4 < (1 << 22)


def bwd_flag_offset(H: int, W: int, P: int) -> int:
    """Byte offset of the fallback flag in mpiv_render_backward's workspace (abi.hip
    bwd_layout): 1 after a call whose last view went through the bucket fallback."""
    return 2 * 64 * 8  # the two pair counters (64 slots of 8 B each) precede it (round 4 layout)


def render_train(rgba_layers: torch.Tensor, homs: torch.Tensor):
    """The forward for training: (frames [B,H,W,3], checkpoints [B,ceil(P/8),H,W,4]) from
    mpiv_render_train -- frames bit-identical to render() -- or (render(), None) when the
    layout is not read in place (a broadcast batch renders from one packed copy instead)."""
    dev = _dev(rgba_layers)
    B, H, W, P, _ = rgba_layers.shape
    if homs.shape[0] != B or homs.shape[1] != P:
        raise RuntimeError(f"shape mismatch: MPI batch/planes {B}/{P} vs poses/planes {homs.shape[0]}/{homs.shape[1]}")
    if (B > 1 and rgba_layers.stride(0) == 0) or not chunk_layout_ok(rgba_layers) or \
            4 * 64 * 9 * 16 + P * 36 > _CHUNK_LDS:
        return render(rgba_layers, homs), None
    h = _up(homs, dev)
    out = torch.empty((B, H, W, 3), device=dev, dtype=torch.float32)
    ckpt = torch.empty((B, (P + 7) // 8, H, W, 4), device=dev, dtype=torch.float32)
    _call("mpiv_render_train", rgba_layers, _strides(rgba_layers), B, H, W, P, h, out, ckpt, _stream(dev))
    return out, ckpt


# MPIV_BWD_MIN_WS=1: render_backward allocates the smallest workspace (plane groups: config 4
# 1.3 GB instead of 3.0, bit-identical gradients, a few percent slower)
BWD_MIN_WS = os.environ.get("MPIV_BWD_MIN_WS") == "1"

# MPIV_BWD_CHECK=1: every render_backward reads the fallback's abort count back (one stream
# synchronisation per call) and raises if a view's gradient was NaN-filled (render_bwd.hip)
BWD_CHECK = os.environ.get("MPIV_BWD_CHECK") == "1"


def render_backward_status(workspace: torch.Tensor, H: int, W: int, P: int) -> int:
    """Views of the last render_backward on this workspace whose bucket fallback aborted
    (their gradients are NaN); synchronises the current stream (mpiv_render_backward_status)."""
    n = _int(0)
    _call("mpiv_render_backward_status", workspace, H, W, P, ctypes.byref(n), _stream(workspace.device))
    return n.value


_BWD_WS: dict = {}


def _bwd_ws_sizes(L, H: int, W: int, P: int):
    """(minimum, fastest) workspace bytes of mpiv_render_backward for one H x W x P view, memoised."""
    key = (L._name, H, W, P, _DEBUG_GEN)  # (the sizes follow debug options such as bwd_group)
    v = _BWD_WS.get(key)
    if v is None:
        v = _BWD_WS[key] = (L.mpiv_render_backward_workspace_size_min(H, W, P),
                            L.mpiv_render_backward_workspace_size(H, W, P))
    return v


class _AbortMonitor:
    """The default (check=None) render_backward's abort report, surfaced without a synchronisation
    (ADVICE r4): the call runs mpiv_render_backward_watched, whose NaN fill of an aborted view also
    sets the device's page-locked, device-mapped abort flag (mpiv_render_backward_abort_flag) from the
    device; the next default render_backward (or render_backward_raise_pending) reads the flag on the
    host -- a memory read, no copy, event or synchronisation (round 5's stream-ordered copy and event
    cost ~30 us per call) -- and raises.  So an aborted fallback (never expected: render_bwd.hip) fails
    the training loop at the latest one step later instead of silently feeding NaN gradients to the
    optimiser."""

    def __init__(self, dev, L):
        self.dev = dev
        ptr = L.mpiv_render_backward_abort_flag(dev.index if dev.index is not None else torch.cuda.current_device())
        if not ptr:
            raise RuntimeError("mpiv_render_backward_abort_flag: no page-locked abort flag for " + str(dev))
        self.flag = ctypes.cast(ptr, ctypes.POINTER(ctypes.c_int))

    def raise_completed(self, wait: bool = False):
        if wait:
            torch.cuda.synchronize(self.dev)
        if self.flag[0]:
            self.flag[0] = 0
            raise RuntimeError("mpiv_render_backward: the bucket fallback aborted on a view of an earlier backward "
                               "(its gradient was NaN)")


_ABORTS: dict = {}


def render_backward_raise_pending(dev=None) -> None:
    """Wait for every earlier default render_backward on `dev` (all devices if None) and raise if
    any of them NaN-filled a view (the check the next call would make)."""
    for (d, _), mon in list(_ABORTS.items()):
        if dev is None or d == torch.device(dev):
            mon.raise_completed(wait=True)


def render_backward(rgba_layers: torch.Tensor, homs: torch.Tensor, dout: torch.Tensor,
                    workspace: torch.Tensor | None = None, ckpt: torch.Tensor | None = None,
                    check: bool | None = None) -> torch.Tensor:
    """d(mpi_render_view_torch)/d(rgba_layers): rgba_layers [B,H,W,P,4] (read in place when
    its planes are contiguous per pixel, incl. a stride-0 broadcast batch; other layouts
    are made contiguous first), homs [B,P,9] (the forward's), dout [B,H,W,3] ->
    [B,H,W,P,4] contiguous, one gradient per view (a broadcast input's views are summed
    by autograd's expand backward, as in the reference).  Bit-exact to the reference's
    CPU autograd (render_bwd.hip).  ckpt: render_train()'s checkpoints of the same views
    (skips recomputing the forward composite).  check (default MPIV_BWD_CHECK): read the
    fallback's abort count back and raise if any view aborted (costs a synchronisation); left at
    None without MPIV_BWD_CHECK, the count is read back asynchronously and a later call raises
    (_AbortMonitor); False: not watched at all."""
    dev = _dev(rgba_layers, dout)
    B, H, W, P, _ = rgba_layers.shape
    if tuple(dout.shape) != (B, H, W, 3):
        raise RuntimeError(f"grad_output must be [{B},{H},{W},3], got {tuple(dout.shape)}")
    src = rgba_layers if bwd_layout_ok(rgba_layers) else rgba_layers.contiguous()
    L = load()
    # a caller's workspace of at least the minimum (plane groups, render_bwd.hip); our own: the
    # one-group size (the fastest schedule) unless MPIV_BWD_MIN_WS=1
    need, full = _bwd_ws_sizes(L, H, W, P)
    ws = workspace if workspace is not None else torch.empty(need if BWD_MIN_WS else full, dtype=torch.uint8,
                                                             device=dev)
    if ws.dtype != torch.uint8 or not ws.is_contiguous() or ws.numel() < need or ws.device != dev:
        raise RuntimeError(f"workspace must be a contiguous uint8 tensor of >= {need} bytes on {dev}")
    grad = torch.empty((B, H, W, P, 4), device=dev, dtype=torch.float32)
    h = _up(homs.reshape(B, P, 9), dev)
    dout = dout.contiguous()
    if ckpt is not None and (tuple(ckpt.shape) != (B, (P + 7) // 8, H, W, 4) or not ckpt.is_contiguous()
                             or ckpt.device != dev or ckpt.dtype != torch.float32):
        raise RuntimeError(f"ckpt must be render_train()'s contiguous [{B},{(P + 7) // 8},{H},{W},4] tensor")
    watch = check is None and not BWD_CHECK
    if watch:
        # (one flag per device and library: the A/B build, when a test selects it, has its own)
        key = (dev, L._name)
        mon = _ABORTS.get(key)
        if mon is None:
            mon = _ABORTS.setdefault(key, _AbortMonitor(dev, L))
        mon.raise_completed()  # an earlier call's abort, read without waiting
    _call("mpiv_render_backward_watched" if watch else "mpiv_render_backward", src, _strides(src), B, H, W, P, h, dout,
          ckpt, grad, ws, ws.numel(), _stream(dev))
    if BWD_CHECK if check is None else check:
        n = render_backward_status(ws, H, W, P)
        if n:
            raise RuntimeError(f"mpiv_render_backward: the bucket fallback aborted on {n} of {B} views "
                               "(their gradients are NaN)")
    return grad


class RenderFunction(torch.autograd.Function):
    """Autograd node of the fused render: forward = render(), backward =
    render_backward() (w.r.t. rgba_layers; homographies come from poses and
    intrinsics, which the reference's training never differentiates)."""

    @staticmethod
    def forward(ctx, rgba_layers, homs):
        ctx.homs = homs
        if ctx.needs_input_grad[0]:  # keep the composite checkpoints for the backward
            out, ckpt = render_train(rgba_layers, homs)
            ctx.save_for_backward(rgba_layers, ckpt)
            return out
        ctx.save_for_backward(rgba_layers, None)
        return render(rgba_layers, homs)

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        rgba_layers, ckpt = ctx.saved_tensors
        grad = render_backward(rgba_layers, ctx.homs, dout, ckpt=ckpt) if ctx.needs_input_grad[0] else None
        return grad, None


# ---------------------------------------------------------------------------
# MPI assembly from the network output (notebook mpi_from_net_output)
# ---------------------------------------------------------------------------

def _net_args(mpi_pred: torch.Tensor, fg: torch.Tensor, P: int):
    dev = _dev(mpi_pred, fg)
    if mpi_pred.dim() != 4 or mpi_pred.shape[1] != 2 * P + 3:
        raise RuntimeError(f"mpi_pred must be [B, 2*{P}+3, H, W], got {tuple(mpi_pred.shape)}")
    B, _, H, W = mpi_pred.shape
    if tuple(fg.shape) != (B, H, W, 3):
        raise RuntimeError(f"ref_img must be [{B},{H},{W},3], got {tuple(fg.shape)}")
    return dev, B, H, W


def assemble_mpi(mpi_pred: torch.Tensor, fg: torch.Tensor, P: int) -> torch.Tensor:
    """[B,2P+3,H,W] prediction + [B,H,W,3] reference image -> MPI [B,H,W,P,4]."""
    dev, B, H, W = _net_args(mpi_pred, fg, P)
    out = torch.empty((B, H, W, P, 4), device=dev, dtype=torch.float32)
    _call("mpiv_assemble_mpi", mpi_pred, _strides(mpi_pred), fg, _strides(fg), B, H, W, P, out, _stream(dev))
    return out


def assemble_mpi_sampled(mpi_pred: torch.Tensor, fg: torch.Tensor, P: int, homs: torch.Tensor) -> torch.Tensor:
    """assemble_mpi for the backward of a render with homs [B,P,9] only: texel rows no output pixel
    of that render can sample are left unwritten (mpiv_assemble_mpi_sampled)."""
    dev, B, H, W = _net_args(mpi_pred, fg, P)
    h = _up(homs.reshape(B, P, 9), dev)
    out = torch.empty((B, H, W, P, 4), device=dev, dtype=torch.float32)
    _call("mpiv_assemble_mpi_sampled", mpi_pred, _strides(mpi_pred), fg, _strides(fg), B, H, W, P, h, out,
          _stream(dev))
    return out


def assemble_mpi_packed(mpi_pred: torch.Tensor, fg: torch.Tensor, P: int, b: int,
                        out: torch.Tensor | None = None) -> torch.Tensor:
    """Batch element b of the assembled MPI, straight into the packed layout [P,H+4,W+4,4]."""
    dev, B, H, W = _net_args(mpi_pred, fg, P)
    if not 0 <= b < B:
        raise IndexError(f"batch index {b} out of range for {B}")
    packed = torch.empty(packed_shape(H, W, P), device=dev, dtype=torch.float32) if out is None else \
        _check_out(out, packed_shape(H, W, P), dev, "assemble_mpi_packed")
    _call("mpiv_assemble_mpi_packed", mpi_pred, _strides(mpi_pred), fg, _strides(fg), b, H, W, P, packed,
          _stream(dev))
    return packed


def render_net_output(mpi_pred: torch.Tensor, fg: torch.Tensor, P: int, homs: torch.Tensor) -> torch.Tensor:
    """Frames [B,H,W,3] of the MPIs assembled from [B,2P+3,H,W] + [B,H,W,3], view b from
    batch element b with homs [B,P,9], in one kernel (render_netout_kernel); bit-identical
    to render(assemble_mpi(...), homs)."""
    dev, B, H, W = _net_args(mpi_pred, fg, P)
    h = _up(homs.reshape(B, P, 9), dev)
    out = torch.empty((B, H, W, 3), device=dev, dtype=torch.float32)
    _call("mpiv_render_net_output", mpi_pred, _strides(mpi_pred), fg, _strides(fg), B, H, W, P, h, out,
          _stream(dev))
    return out


def netout_ckpt_ok(H: int, W: int, P: int) -> bool:
    """True when the fused training forward keeps composite checkpoints: exactly when
    render_train() would for the assembled (contiguous) MPI -- the backward reads it in place."""
    return H >= 2 and W >= 2 and 4 * 64 * 9 * 16 + P * 36 <= _CHUNK_LDS


def render_net_output_train(mpi_pred: torch.Tensor, fg: torch.Tensor, P: int, homs: torch.Tensor):
    """The fused net-output render's training forward: (frames [B,H,W,3], checkpoints
    [B,ceil(P/8),H,W,4]) -- the frames of render_net_output() and the checkpoints render_train()
    writes for the assembled MPI, bit for bit (mpiv_render_net_output_train); (frames, None) where
    render_train() keeps none."""
    dev, B, H, W = _net_args(mpi_pred, fg, P)
    if not netout_ckpt_ok(H, W, P):
        return render_net_output(mpi_pred, fg, P, homs), None
    h = _up(homs.reshape(B, P, 9), dev)
    out = torch.empty((B, H, W, 3), device=dev, dtype=torch.float32)
    ckpt = torch.empty((B, (P + 7) // 8, H, W, 4), device=dev, dtype=torch.float32)
    _call("mpiv_render_net_output_train", mpi_pred, _strides(mpi_pred), fg, _strides(fg), B, H, W, P, h, out, ckpt,
          _stream(dev))
    return out, ckpt


class NetOutputRenderFunction(torch.autograd.Function):
    """Autograd node of the fused assembly + render (the training losses' two lines, ipynb cell 12
    L7-11 / L38-42: mpi_from_net_output then mpi_render_view_torch) that never keeps the
    [B,H,W,P,4] MPI between forward and backward.  Forward: render_netout_kernel with the
    composite checkpoints (saves pred, ref image, checkpoints: (2P+3+3)*4 + ceil(P/8)*16 B per pixel
    instead of the MPI's P*16 + the checkpoints).  Backward: the MPI re-assembled (assemble.hip; the
    texel rows the render samples only, mpiv_assemble_mpi_sampled),
    render_backward with those checkpoints, the assembly adjoint -- the two-step chain's own
    kernels in its order, so d pred / d ref_img are bit-identical to it and to the reference's
    autograd (tests/golden/netout_train.npz)."""

    @staticmethod
    def forward(ctx, mpi_pred, fg, homs, P):
        ctx.P = P
        ctx.homs = homs
        out, ckpt = render_net_output_train(mpi_pred, fg, P, homs)
        ctx.save_for_backward(mpi_pred, fg, ckpt)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        mpi_pred, fg, ckpt = ctx.saved_tensors
        if not (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]):
            return None, None, None, None
        # only the texel rows the render samples (round 6): the chain reads no other
        rgba = assemble_mpi_sampled(mpi_pred, fg, ctx.P, ctx.homs)
        drgba = render_backward(rgba, ctx.homs, dout, ckpt=ckpt)
        del rgba  # the re-assembled MPI lives only for the chain
        res = assemble_mpi_backward(drgba, mpi_pred, fg, ctx.P, want_dfg=ctx.needs_input_grad[1])
        dpred, dfg = res if ctx.needs_input_grad[1] else (res, None)
        return (dpred if ctx.needs_input_grad[0] else None), dfg, None, None


def assemble_mpi_backward(drgba: torch.Tensor, mpi_pred: torch.Tensor, fg: torch.Tensor, P: int,
                          want_dfg: bool = False):
    """d pred [B,2P+3,H,W] (and, with want_dfg, (d pred, d fg [B,H,W,3])) for d rgba."""
    dev, B, H, W = _net_args(mpi_pred, fg, P)
    _dev(drgba)
    if tuple(drgba.shape) != (B, H, W, P, 4):
        raise RuntimeError(f"grad must be [{B},{H},{W},{P},4], got {tuple(drgba.shape)}")
    dpred = torch.empty((B, 2 * P + 3, H, W), device=dev, dtype=torch.float32)
    dfg = torch.empty((B, H, W, 3), device=dev, dtype=torch.float32) if want_dfg else None
    _call("mpiv_assemble_mpi_backward", drgba, _strides(drgba), mpi_pred, _strides(mpi_pred), fg, _strides(fg),
          B, H, W, P, dpred, dfg, _stream(dev))
    return (dpred, dfg) if want_dfg else dpred


class AssembleFunction(torch.autograd.Function):
    """Autograd node of the assembly: gradients w.r.t. the network prediction and, when
    it requires grad, the reference image (both bit-exact to the notebook's autograd)."""

    @staticmethod
    def forward(ctx, mpi_pred, fg, P):
        ctx.save_for_backward(mpi_pred, fg)
        ctx.P = P
        return assemble_mpi(mpi_pred, fg, P)

    @staticmethod
    @once_differentiable
    def backward(ctx, drgba):
        mpi_pred, fg = ctx.saved_tensors
        if not (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]):
            return None, None, None
        res = assemble_mpi_backward(drgba, mpi_pred, fg, ctx.P, want_dfg=ctx.needs_input_grad[1])
        dpred, dfg = res if ctx.needs_input_grad[1] else (res, None)
        return (dpred if ctx.needs_input_grad[0] else None), dfg, None


# ---------------------------------------------------------------------------
# plane sweep / inverse warp
# ---------------------------------------------------------------------------

_DEPTHS_DEV: dict = {}


def _depths_on(depth_planes, dev, sid=None) -> torch.Tensor:
    """The sweep depths as a contiguous fp32 tensor on `dev`.  The reference iterates
    `for depth in depth_planes` and adds each to an fp32 zero map (utils.py:466-467), so a
    list of floats and a tensor (the notebook passes torch.Tensor(inv_depths(...)).to(device),
    ipynb cell 8 L73) both mean their values rounded to fp32.  A device tensor is used where
    it is (no per-element reads back to the host); a list is uploaded once per distinct value
    list and device (memoised)."""
    if isinstance(depth_planes, torch.Tensor):
        return depth_planes.detach().to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    # keyed on the values (numbers hash and compare by value, so a list of Python or numpy
    # floats finds the same entry), the device and the stream: the copy is allocated on (and
    # its memory, once evicted, reused in the order of) the stream that made it, so each stream
    # reads only its own copy
    if sid is None:
        sid = torch.cuda.current_stream(dev).cuda_stream
    key = (tuple(depth_planes), dev.index, sid)
    d = _DEPTHS_DEV.get(key)
    if d is None:
        if len(_DEPTHS_DEV) >= 64:
            _DEPTHS_DEV.clear()
        d = torch.tensor([float(x) for x in key[0]], dtype=torch.float32).to(dev)
        _DEPTHS_DEV[key] = d
    return d


def _require_depths(depth_planes) -> None:
    # the reference concatenates one slice per depth (utils.py:466-470): no depths is
    # torch.cat.s ValueError, raised here before anything is launched
    if len(depth_planes) == 0:
        raise ValueError("torch.cat(): expected a non-empty list of Tensors")


def plane_sweep(img: torch.Tensor, depth_planes, ki: torch.Tensor, proj: torch.Tensor, tgt_h: int,
                tgt_w: int) -> torch.Tensor:
    """[B,Hs,Ws,C] -> PSV [B,tgt_h,tgt_w,D*C] in one launch (mpiv_plane_sweep): C <= 4 through
    the depth-per-lane LDS kernel reading the source in place (any strides, no padded
    copy), C > 4 through the generic strided kernel."""
    _require_depths(depth_planes)
    dev = _dev(img)
    B, Hs, Ws, C = img.shape
    dd = _depths_on(depth_planes, dev)
    D = dd.shape[0]
    out = torch.empty((B, tgt_h, tgt_w, D * C), device=dev, dtype=torch.float32)
    kid, projd = _up(ki, dev), _up(proj, dev)
    _call("mpiv_plane_sweep", img, _strides(img), B, Hs, Ws, C, kid, projd, dd, D, tgt_h, tgt_w, out, _stream(dev))
    return out


_PROJ_SCRATCH: dict = {}
_STRIDES4: dict = {}


def plane_sweep_pose(img: torch.Tensor, depth_planes, ki: torch.Tensor, Ks: torch.Tensor, pose: torch.Tensor,
                     tgt_h: int, tgt_w: int, stream=None) -> torch.Tensor:
    """plane_sweep with proj = K4_src @ pose formed on the device in the same call
    (mpiv_plane_sweep_pose): img [B,Hs,Ws,C] or, unbatched, [Hs,Ws,C] (plane_sweep_torch_one's
    call: B = 1, the result still [1,...]); ki [B,9] on the device, Ks [3,3] (one camera) or
    [B,3,3] with 3x3 blocks contiguous, pose [B,4,4] (or [4,4]) contiguous fp32 on the device.
    The [B,16] proj lands in a scratch buffer kept per device and stream (reused in stream
    order).  The notebook's dataset calls this once per sample at 224x224x10, where the kernel
    is ~12 us, so the host path is kept to a handful of torch calls."""
    _require_depths(depth_planes)
    dev = _dev(img, Ks, pose)
    if img.dim() == 3:
        Hs, Ws, C = img.shape
        B = 1
        st = img.stride()
        st = (Hs * st[0], st[0], st[1], st[2])
    else:
        B, Hs, Ws, C = img.shape
        st = img.stride()
    cst = _STRIDES4.get(st)
    if cst is None:
        if len(_STRIDES4) >= 256:
            _STRIDES4.clear()
        cst = _STRIDES4[st] = (ctypes.c_int64 * 4)(*st)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    sid = stream.cuda_stream
    dd = _depths_on(depth_planes, dev, sid)
    D = dd.shape[0]
    key = (dev.index, sid)
    scratch = _PROJ_SCRATCH.get(key)
    if scratch is None or scratch.numel() < B * 16:
        scratch = _PROJ_SCRATCH[key] = torch.empty(max(B, 8) * 16, device=dev, dtype=torch.float32)
    ks_b = 0 if Ks.dim() == 2 else Ks.stride(0)
    out = torch.empty((B, tgt_h, tgt_w, D * C), device=dev, dtype=torch.float32)
    _call("mpiv_plane_sweep_pose", img, cst, B, Hs, Ws, C, ki, Ks, ks_b, pose, scratch, dd, D, tgt_h, tgt_w,
          out, _vp(sid))
    return out


def plane_sweep_padded(img: torch.Tensor, depth_planes, ki: torch.Tensor, proj: torch.Tensor, tgt_h: int,
                       tgt_w: int) -> torch.Tensor:
    """plane_sweep through a padded 16-B texel copy of the source (mpiv_pad_texels +
    mpiv_plane_sweep_padded; C <= 4): the pixel-per-lane / tile / grouped kernels' input
    (A/B and tests)."""
    _require_depths(depth_planes)
    dev = _dev(img)
    B, Hs, Ws, C = img.shape
    dd = _depths_on(depth_planes, dev)
    D = dd.shape[0]
    out = torch.empty((B, tgt_h, tgt_w, D * C), device=dev, dtype=torch.float32)
    img4 = pad_texels(img)
    _call("mpiv_plane_sweep_padded", img4, B, Hs, Ws, C, _up(ki, dev), _up(proj, dev), dd, D, tgt_h,
          tgt_w, out, _stream(dev))
    return out


def pad_texels(img: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """[B,Hs,Ws,C<=4] (any strides) -> [B,Hs+4,Ws+4,4] 16-B texels with a 2-texel zero
    border (mpiv_pad_texels layout)."""
    dev = _dev(img)
    B, Hs, Ws, C = img.shape
    shape = (B, Hs + 4, Ws + 4, 4)
    if out is None:
        out = torch.empty(shape, device=dev, dtype=torch.float32)
    elif tuple(out.shape) != shape or not out.is_contiguous():
        raise RuntimeError(f"pad_texels: out must be a contiguous {shape} tensor")
    _call("mpiv_pad_texels", img, _strides(img), B, Hs, Ws, C, out, _stream(dev))
    return out


def preprocess(image: torch.Tensor) -> torch.Tensor:
    dev = _dev(image)
    src = image.contiguous()
    out = torch.empty_like(src)
    _call("mpiv_preprocess", src, src.numel(), out, _stream(dev))
    return out


def deprocess_u8(image: torch.Tensor) -> torch.Tensor:
    dev = _dev(image)
    src = image.contiguous()
    out = torch.empty(src.shape, device=dev, dtype=torch.uint8)
    _call("mpiv_deprocess_u8", src, src.numel(), out, _stream(dev))
    return out


def network_input(ref_image, psv_src_images, rel_poses, depth_planes, intrinsics) -> torch.Tensor:
    """format_network_input_torch: [B,H,W,3] ref + S PSVs of the 3-channel slices of
    psv_src_images, each swept directly into its channel range of one output."""
    from ._host import psv_matrices
    if len(rel_poses):
        _require_depths(depth_planes)
    dev = _dev(ref_image, psv_src_images)
    B, H, W, _ = ref_image.shape
    S = len(rel_poses)
    dd = _depths_on(depth_planes, dev) if S else None
    D = dd.shape[0] if S else len(depth_planes)
    Ctot = 3 + S * D * 3
    out = torch.empty((B, H, W, Ctot), device=dev, dtype=torch.float32)
    out[..., :3].copy_(ref_image)  # the concat's first slice is a plain copy (utils.py:491)
    for i, pose in enumerate(rel_poses):
        src = psv_src_images[:, :, :, i * 3:(i + 1) * 3]  # a strided channel slice, read in place
        ki, proj = psv_matrices(intrinsics, intrinsics, pose, pin=True)
        _call("mpiv_plane_sweep_into", src, _strides(src), B, H, W, 3, _up(ki, dev), _up(proj, dev), dd, D, H, W,
              out[..., 3 + i * D * 3:], H * W * Ctot, Ctot, _stream(dev))
    return out


def inverse_warp_depthmap(img, depth, ki, proj, tgt_h, tgt_w):
    dev = _dev(img, depth)
    B, Hs, Ws, C = img.shape
    if tuple(depth.shape) != (B, tgt_h, tgt_w):
        raise RuntimeError(f"depth must be [{B},{tgt_h},{tgt_w}], got {tuple(depth.shape)}")
    out = torch.empty((B, tgt_h, tgt_w, C), device=dev, dtype=torch.float32)
    _call("mpiv_inverse_warp", img, _strides(img), B, Hs, Ws, C, _up(ki, dev), _up(proj, dev),
          depth, _strides(depth), tgt_h, tgt_w, out, _stream(dev))
    return out


# ---------------------------------------------------------------------------
# sampler / compositor primitives
# ---------------------------------------------------------------------------

def bilinear_sample(imgs: torch.Tensor, coords: torch.Tensor, channels_last_out: bool) -> torch.Tensor:
    """channels_last_out=False: bilinear_wrapper_torch semantics ([..., Hs, Ws, C] ->
    [..., C, Ht, Wt]); True: resampler_wrapper_torch ([N,H,W,C] -> [N,H',W',C])."""
    dev = _dev(imgs, coords)
    if channels_last_out:
        if imgs.dim() != 4 or coords.dim() != 4:
            raise RuntimeError("resampler_wrapper_torch expects imgs [N,H,W,C] and coords [N,H,W,2]")
        lead = [imgs.shape[0]]
        im4 = imgs
        co4 = coords
    else:
        lead = list(imgs.shape[:-3])
        n = lead[0]  # IndexError for 3-d input, like the reference (utils.py:117)
        for s in lead[1:]:
            n *= s
        im4 = imgs.reshape([n] + list(imgs.shape[-3:]))
        co4 = coords.reshape([n] + list(coords.shape[-3:]))
    N, Hi, Wi, C = im4.shape
    if co4.shape[0] != N or co4.shape[-1] != 2:
        raise RuntimeError(f"grid_sample: coords {tuple(coords.shape)} do not match images {tuple(imgs.shape)}")
    Ho, Wo = co4.shape[1], co4.shape[2]
    if channels_last_out:
        out = torch.empty((N, Ho, Wo, C), device=dev, dtype=torch.float32)
        ost = _strides(out, (0, 3, 1, 2))
    else:
        out = torch.empty((N, C, Ho, Wo), device=dev, dtype=torch.float32)
        ost = _strides(out)
    _call("mpiv_grid_sample", im4, _strides(im4, (0, 3, 1, 2)), N, C, Hi, Wi, co4, _strides(co4), Ho, Wo,
          out, ost, _stream(dev))
    if channels_last_out:
        return out
    return out.reshape(lead + [C, Ho, Wo])


def _flat_pixels(t: torch.Tensor):
    """(pixel_stride, channel_stride) if the leading dims of t [..., 4] collapse to one
    uniform pixel stride, else None."""
    ps = t.stride(-2) if t.dim() >= 2 else 0
    expect = ps
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] != 1 and t.stride(d) != expect:
            return None
        expect *= t.shape[d]
    return ps, t.stride(-1)


def over_composite(rgbas) -> torch.Tensor:
    rgbas = list(rgbas)
    if not rgbas:
        raise UnboundLocalError("over_composite: empty list")  # the reference fails the same way
    dev = _dev(*rgbas)
    shape = rgbas[0].shape
    if shape[-1] != 4:
        raise RuntimeError(f"over_composite expects RGBA layers, got {tuple(shape)}")
    layers = []
    for t in rgbas:
        if t.shape != shape:
            raise RuntimeError(f"over_composite: layer shapes differ {tuple(shape)} vs {tuple(t.shape)}")
        layers.append(t)
    # one (pixel stride, channel stride) pair must describe every layer; else copy
    if None in {_flat_pixels(t) for t in layers} or len({_flat_pixels(t) for t in layers}) != 1:
        layers = [t.contiguous() for t in layers]
    ps, cs = _flat_pixels(layers[0])
    n = layers[0].numel() // 4
    ptrs = torch.tensor([t.data_ptr() for t in layers], dtype=torch.int64).to(dev)
    out = torch.empty(tuple(shape[:-1]) + (3,), device=dev, dtype=torch.float32)
    _call("mpiv_over_composite", ptrs, len(layers), n, ps, cs, out, _stream(dev))
    # temporaries (pointer table, contiguous copies) may be freed now: the caching
    # allocator only hands their memory to later work on this same stream
    return out


# ---------------------------------------------------------------------------
# geometry helpers
# ---------------------------------------------------------------------------

def transform_points(points: torch.Tensor, homography: torch.Tensor) -> torch.Tensor:
    dev = _dev(points, homography)
    hshape = list(homography.shape)
    M = 1
    for s in hshape[:-2]:
        M *= s
    pts = points.reshape(hshape[:-2] + [-1, 3]).contiguous()
    n = pts.shape[-2]
    out = torch.empty_like(pts)
    _call("mpiv_transform_points", pts, M, n, homography.reshape(M, 9).contiguous(), out,
          _stream(dev))
    return out.reshape(points.shape)


def normalize_homogeneous(points: torch.Tensor) -> torch.Tensor:
    dev = _dev(points)
    k = points.shape[-1] - 1
    if k < 1:
        raise RuntimeError("normalize_homogeneous_torch needs at least 2 coordinates")
    work = points if points.is_contiguous() else points.contiguous()
    out = torch.empty(tuple(points.shape[:-1]) + (k,), device=dev, dtype=torch.float32)
    _call("mpiv_normalize_homogeneous", work, work.numel() // (k + 1), k, out, _stream(dev))
    if work is not points:  # keep the reference's in-place w update visible
        points.copy_(work)
    return out


def pixel2cam(depth, pixel_coords, intrinsics, is_homogeneous=True):
    dev = _dev(depth, pixel_coords)
    B, H, W = depth.shape
    n = H * W
    from ._host import _cpu32
    ki = torch.inverse(_cpu32(intrinsics)).reshape(B, 9)
    rows = 4 if is_homogeneous else 3
    cam = torch.empty((B, rows, H, W), device=dev, dtype=torch.float32)
    _call("mpiv_pixel2cam", depth.contiguous(), pixel_coords.reshape(B, 3, n).contiguous(),
          _up(ki, dev), B, n, int(bool(is_homogeneous)), cam, _stream(dev))
    return cam


def cam2pixel(cam_coords, proj):
    dev = _dev(cam_coords, proj)
    B, _, H, W = cam_coords.shape
    n = H * W
    out = torch.empty((B, H, W, 2), device=dev, dtype=torch.float32)
    _call("mpiv_cam2pixel", cam_coords.reshape(B, 4, n).contiguous(), proj.reshape(B, 16).contiguous(), B,
          n, out, _stream(dev))
    return out


def warp_planes(imgs: torch.Tensor, pixel_coords_trg: torch.Tensor, hom: torch.Tensor) -> torch.Tensor:
    """transform_plane_imgs_torch: imgs [..., Hs, Ws, C], target points [..., Ht, Wt, 3],
    hom [..., 3, 3] -> [..., C, Ht, Wt]."""
    dev = _dev(imgs, pixel_coords_trg)
    hshape = list(hom.shape)
    M = 1
    for s in hshape[:-2]:
        M *= s
    Ht, Wt = pixel_coords_trg.shape[-3], pixel_coords_trg.shape[-2]
    pts = pixel_coords_trg.reshape(M, Ht * Wt, 3).contiguous()
    coords = torch.empty((M, Ht, Wt, 2), device=dev, dtype=torch.float32)
    _call("mpiv_plane_coords", pts, M, Ht * Wt, _up(hom.reshape(M, 9), dev), Ht, Wt, coords,
          _stream(dev))
    return bilinear_sample(imgs, coords.reshape(list(pixel_coords_trg.shape[:-1]) + [2]), channels_last_out=False)

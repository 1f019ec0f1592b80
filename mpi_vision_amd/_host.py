"""Host-side 3x3 / 4x4 setup for the render and plane-sweep kernels.

These matrices are tiny (P*B 3x3 homographies, B 3x3 + 4x4 PSV matrices) but
their exact fp32 bits decide whether the kernels land within 1e-5 of the
reference (a float64-derived H breaks 1e-5 on ~1.4% of pixels).
So they are computed with torch-CPU fp32 ops in the reference's association
order -- the same ATen kernels the reference itself calls -- and then uploaded
once per call (P*B*36 bytes).
"""
from __future__ import annotations

import weakref

import torch

_CPU = torch.device("cpu")
_F32 = torch.float32


def _cpu32(x: torch.Tensor) -> torch.Tensor:
    return x.detach().to(device=_CPU, dtype=_F32)


def divide_safe(num: torch.Tensor, den: torch.Tensor) -> torch.Tensor:
    """utils.py:35-39: den == 0 -> den + 1e-8 (fp32), then num / den."""
    den = den.to(_F32)
    den = den + 1e-8 * (den == 0)
    return num.to(_F32) / den


def inv_homography(k_s, k_t, rot, t, n_hat, a):
    """utils.py:44-67, same op order:
        denom     = a - (n_hat @ R^T) @ t
        numerator = ((R^T @ t) @ n_hat) @ R^T
        H         = (k_s @ (R^T + numerator / denom)) @ inverse(k_t)
    Runs on the inputs' device (the render path calls it with CPU tensors)."""
    rot_t = rot.transpose(-2, -1)
    k_t_inv = torch.inverse(k_t)
    denom = a - torch.matmul(torch.matmul(n_hat, rot_t), t)
    numerator = torch.matmul(torch.matmul(torch.matmul(rot_t, t), n_hat), rot_t)
    return torch.matmul(torch.matmul(k_s, rot_t + divide_safe(numerator, denom)), k_t_inv)


_KINV_CACHE: dict = {}


def _inverse_cached(K: torch.Tensor) -> torch.Tensor:
    """torch.inverse(K) for fp32 CPU K [B,3,3] AS LAID OUT (contiguous [B,3,3] result),
    memoised on K's exact bits and its size / strides (intrinsics rarely change along a camera
    path; LAPACK is ~10 us of the host path).  The layout is part of the key because torch's
    CPU inverse returns different bits for the same values in a different layout (a stride-0
    batch, F-ordered or sliced blocks: tests/test_kstride.py).  A contiguous batch is inverted
    element by element, so the result equals the reference's inverse of its [P,B,3,3] repeat
    element for element (tests/test_host.py)."""
    key = (tuple(K.shape), tuple(K.stride()), K.contiguous().numpy().tobytes())
    kinv = _KINV_CACHE.get(key)
    if kinv is None:
        if len(_KINV_CACHE) >= 256:
            _KINV_CACHE.clear()
        kinv = torch.inverse(K).contiguous()
        _KINV_CACHE[key] = kinv
    return kinv


def cpu32_like(x: torch.Tensor) -> torch.Tensor:
    """fp32 CPU tensor with x's values AND x's size and strides (stride-0 broadcasts, F-ordered
    or sliced blocks kept).  `.cpu()` materialises a non-dense tensor, which would change what
    torch.inverse returns; here the storage span x covers is copied once and re-viewed with x's
    strides."""
    x = x.detach()
    if x.device.type == "cpu" and x.dtype == _F32:
        return x
    if x.numel() == 0:
        return torch.empty(x.shape, dtype=_F32)
    span = 1 + sum((n - 1) * st for n, st in zip(x.shape, x.stride()))
    flat = torch.as_strided(x, (span,), (1,), x.storage_offset()).to(device=_CPU, dtype=_F32)
    return torch.as_strided(flat, x.shape, x.stride())


def psv_inverse(K: torch.Tensor, batch: int) -> torch.Tensor:
    """Ki = inverse(K_tgt) [batch, 3, 3] (contiguous) as pixel2cam_torch computes it:
    `torch.inverse(intrinsics)` on the CALLER's tensor (utils.py:370, from :428 / :747), so on
    a CPU copy with the caller's strides (cpu32_like), not a materialised one -- a shared camera
    passed as K[None].expand(B,3,3) inverts to other bits than its .contiguous() copy, and the
    PSV moves by up to ~6e-5 with it (tests/golden/kstride.npz, tools/gen_goldens_kstride.py).
    The unbatched _one / _one2 calls pass intrinsics.unsqueeze(0) (utils.py:530, :795), which this
    receives as [1,3,3].  A single camera for a larger batch ([3,3] or [1,3,3], which the
    reference's torch.cat rejects, utils.py:433) is inverted once as given and broadcast."""
    Kc = cpu32_like(K)
    if Kc.dim() == 2:
        Kc = Kc.unsqueeze(0)
    kinv = _inverse_cached(Kc)
    if kinv.shape[0] != batch:
        kinv = kinv.expand(batch, 3, 3).contiguous()
    return kinv


_KINV_DEV: dict = {}


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream_id(dev) -> int:
    """The raw handle of dev's current stream (no torch Stream object built: per-call path)."""
    if _raw_stream is not None:
        return _raw_stream(dev.index if dev.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(dev).cuda_stream


def _f32_on(t: torch.Tensor, dev) -> torch.Tensor:
    return t if (t.dtype == _F32 and t.device == dev) else t.to(device=dev, dtype=_F32)


def _kinv_device(intrinsics: torch.Tensor, batch: int, dev, sid=None, psv: bool = False) -> torch.Tensor:
    """inverse(K) [batch,3,3] on `dev` for a device-resident intrinsics tensor, memoised on
    that tensor OBJECT and its version counter (an in-place update bumps it; a new tensor
    is a new object), so a camera path that reuses one intrinsics tensor reads it back to
    the host once.  On a miss: one device-to-host copy of K and LAPACK (torch.inverse, as
    the reference), then the upload.

    psv=False (render): the reference inverts its materialised [P,B,3,3] repeat of K
    (utils.py:225-228 -> :60), so K is inverted contiguous.  psv=True: the caller's own layout
    (psv_inverse, utils.py:370)."""
    try:
        ver = intrinsics._version
    except RuntimeError:  # inference tensors track no version: no memo
        ver = None
    # the stream is part of the key: the copy's memory, once evicted, is reused in the order of
    # the stream that allocated it, so each stream reads only its own copy
    stream = _raw_stream_id(dev) if sid is None else sid
    ent = _KINV_DEV.get((id(intrinsics), psv))
    same = (ver is not None and ent is not None and ent[0]() is intrinsics and ent[1] == ver and ent[2] == batch
            and ent[3].device == dev)
    if same and ent[4] == stream:
        return ent[3]
    if torch.cuda.is_current_stream_capturing():
        # HIP-graph capture (torch.cuda.graph / make_graphed_callables): a device-to-host copy cannot be
        # captured.  The inverse memoised during the warm-up (on another stream) is copied device to
        # device instead -- a captured copy into the graph's own memory pool, so replays never read
        # memory the memo may free.
        if same:
            return ent[3].clone()
        raise RuntimeError("mpi_vision_amd: inverse(intrinsics) is not memoised for this tensor; run the call "
                           "once outside the HIP-graph capture (the warm-up) first")
    if psv:
        kinv = psv_inverse(intrinsics, batch).to(dev)
    else:
        K = _cpu32(intrinsics).expand(batch, 3, 3).contiguous()
        kinv = _inverse_cached(K).to(dev)
    if ver is not None:
        if len(_KINV_DEV) >= 64:
            _KINV_DEV.clear()
        _KINV_DEV[(id(intrinsics), psv)] = (weakref.ref(intrinsics), ver, batch, kinv, stream)
    return kinv


def render_homographies_device(pose: torch.Tensor, depths: torch.Tensor, intrinsics: torch.Tensor,
                               batch: int) -> torch.Tensor:
    """render_homographies for a pose batch that lives on a ROCm device: the same chain
    evaluated there (mpiv_render_homographies_device, bit-identical to the host entry),
    so the render path issues no blocking device-to-host copy of the poses.  Returns a
    [B, P, 9] fp32 tensor on the pose's device."""
    from . import _lib
    dev = pose.device
    pose_d = _f32_on(pose, dev).contiguous()
    d = _f32_on(depths, dev).reshape(-1).contiguous()
    K = _f32_on(intrinsics, dev)
    if tuple(K.shape) != (batch, 3, 3):
        K = K.expand(batch, 3, 3)
    K = K.contiguous()
    kinv = _kinv_device(intrinsics, batch, dev)
    P = d.shape[0]
    H = torch.empty((batch, P, 9), dtype=_F32, device=dev)
    _lib._call("mpiv_render_homographies_device", pose_d, d, K, kinv, batch, P, H, _lib._stream(dev))
    return H


def render_homographies(pose: torch.Tensor, depths: torch.Tensor, intrinsics: torch.Tensor,
                        batch: int, pin: bool = False) -> torch.Tensor:
    """Per-(view, plane) target->source homographies for mpi_render_view_torch
    (utils.py:278-285 -> 255-262 -> 225-229 -> 44-67), as a [B, P, 9] fp32 CPU tensor
    (page-locked with pin=True, ready for an asynchronous upload).

    The chain runs in libmpiv's host code (mpiv_render_homographies): torch's CPU matmul
    of these tiny matrices is plain products summed in ascending k, which the library
    restates exactly; only K^-1 comes from torch.inverse (LAPACK), as in the reference.
    ~35 tiny torch ops (~0.2 ms of dispatch) become one call.  render_homographies_torch
    keeps the op-by-op form (tests compare the two bit for bit)."""
    from . import _lib
    pose = _cpu32(pose).contiguous()
    K = _cpu32(intrinsics).expand(batch, 3, 3).contiguous()
    d = _cpu32(depths).reshape(-1).contiguous()
    P = d.shape[0]
    kinv = _inverse_cached(K)
    H = torch.empty((batch, P, 9), dtype=_F32, pin_memory=pin)
    rc = _lib.load().mpiv_render_homographies(pose.data_ptr(), d.data_ptr(), K.data_ptr(), kinv.data_ptr(),
                                              batch, P, H.data_ptr())
    if rc != 0:
        raise RuntimeError(f"mpiv_render_homographies failed ({rc}): {_lib.load().mpiv_last_error().decode()}")
    return H


def render_homographies_torch(pose: torch.Tensor, depths: torch.Tensor, intrinsics: torch.Tensor,
                              batch: int) -> torch.Tensor:
    """render_homographies with the reference's torch ops, op for op.

    The reference materialises every camera tensor as a contiguous [P, B, ...]
    repeat before the matmul chain (utils.py:225-228, 258).  That matters: on
    stride-0 (expanded) operands torch.matmul folds the batch into one MKL sgemm
    whose FMA rounding differs by up to ~4e-6 in H, so the repeats are kept."""
    pose = _cpu32(pose)
    K = _cpu32(intrinsics)
    P = depths.shape[0]
    d = _cpu32(depths).reshape(P, 1).repeat(1, batch)
    rot = pose[:, :3, :3].unsqueeze(0).repeat(P, 1, 1, 1)
    t = pose[:, :3, 3:].unsqueeze(0).repeat(P, 1, 1, 1)
    n_hat = torch.tensor([0.0, 0.0, 1.0], dtype=_F32).reshape(1, 1, 1, 3).repeat(P, batch, 1, 1)
    a = -d.reshape(P, batch, 1, 1)
    k = K.unsqueeze(0).repeat(P, 1, 1, 1)
    H = inv_homography(k, k, rot, t, n_hat, a)  # [P, B, 3, 3]
    return H.permute(1, 0, 2, 3).reshape(batch, P, 9).contiguous()


def _cpu32_together(*ts: torch.Tensor):
    """fp32 CPU copies of several tensors with ONE device-to-host transfer when any of them
    lives on a device (the PSV drop-in's caller keeps K and the pose on the GPU, ipynb cell 8
    L49-75: one blocking copy instead of three)."""
    if not any(t.device.type != "cpu" for t in ts):
        return [_cpu32(t) for t in ts]
    dev = next(t.device for t in ts if t.device.type != "cpu")
    flat = torch.cat([t.detach().to(device=dev, dtype=_F32).reshape(-1) for t in ts]).cpu()
    out, o = [], 0
    for t in ts:
        n = t.numel()
        out.append(flat[o:o + n].reshape(t.shape))
        o += n
    return out


def psv_matrices(src_intrinsics: torch.Tensor, tgt_intrinsics: torch.Tensor, pose: torch.Tensor, pin: bool = False):
    """Matrices for projective_inverse_warp_torch[2] (utils.py:428-438, 747-757):
        Ki   = inverse(K_tgt)                       [B, 9]
        proj = [[K_src, 0], [0, 0, 0, 1]] @ pose    [B, 16]
    computed on CPU in fp32 with the reference's ops (page-locked with pin=True, ready for
    an asynchronous upload)."""
    kt = tgt_intrinsics.detach()
    if kt.device.type != "cpu" and kt.numel() > 0:
        # the storage span of K_tgt rides in the same device-to-host copy and is
        # re-viewed on the host with the caller's strides (cpu32_like's contract)
        span = 1 + sum((n - 1) * st for n, st in zip(kt.shape, kt.stride()))
        Ks, pose, kflat = _cpu32_together(src_intrinsics, pose,
                                          torch.as_strided(kt, (span,), (1,), kt.storage_offset()))
        kt = torch.as_strided(kflat, kt.shape, kt.stride())
    else:
        Ks, pose = _cpu32_together(src_intrinsics, pose)
    B = pose.shape[0]
    ki = psv_inverse(kt, B)  # the caller's layout (utils.py:370)
    Ks = Ks.expand(B, 3, 3)
    k4 = torch.cat([Ks, torch.zeros(B, 3, 1)], dim=2)
    k4 = torch.cat([k4, torch.tensor([[[0.0, 0.0, 0.0, 1.0]]]).repeat(B, 1, 1)], dim=1)
    proj = torch.matmul(k4, pose)
    ki, proj = ki.reshape(B, 9).contiguous(), proj.reshape(B, 16).contiguous()
    if pin:
        ki, proj = ki.pin_memory(), proj.pin_memory()
    return ki, proj


def psv_ki_device(tgt_intrinsics: torch.Tensor, batch: int, dev, sid=None) -> torch.Tensor:
    """Ki = inverse(K_tgt) [batch, 3, 3] (contiguous: read as [batch, 9]) on dev, memoised per
    intrinsics tensor (_kinv_device), inverted in the caller's layout (psv_inverse)."""
    return _kinv_device(tgt_intrinsics, batch, dev, sid, psv=True)


def device_cameras(src_intrinsics: torch.Tensor, pose: torch.Tensor, batch: int):
    """(Ks, pose) as the device kernels take them: Ks fp32 [3,3] (one camera) or [batch,3,3]
    with contiguous 3x3 blocks, pose fp32 [batch,4,4] contiguous, on the pose's device."""
    dev = pose.device
    Ks = src_intrinsics
    if Ks.dtype != _F32 or Ks.device != dev:
        Ks = Ks.to(device=dev, dtype=_F32)
    if Ks.dim() == 2:
        if not Ks.is_contiguous():
            Ks = Ks.contiguous()
    else:
        Ks = Ks.expand(batch, 3, 3)
        if Ks.stride(1) != 3 or Ks.stride(2) != 1:
            Ks = Ks.contiguous()
    if pose.dtype != _F32:
        pose = pose.to(dtype=_F32)
    if not pose.is_contiguous():
        pose = pose.contiguous()
    return Ks, pose  # [4,4] or [batch,4,4]: the kernel reads batch * 16 floats


def psv_matrices_device(src_intrinsics: torch.Tensor, tgt_intrinsics: torch.Tensor, pose: torch.Tensor,
                        batch: int):
    """psv_matrices for a pose that lives on a ROCm device (the notebook's dataset call keeps
    pose and K in HBM, ipynb cell 8 L49-75): Ki = inverse(K_tgt) memoised on the intrinsics
    tensor object and its version (_kinv_device: one LAPACK inverse per camera, as the
    reference), proj = K4_src @ pose by mpiv_psv_proj_device on the current stream (the host
    entry's restatement, bit-identical).  No device-to-host copy, no page-locked staging.
    Intrinsics [3,3] (one camera for the batch) or [batch,3,3]; pose [batch,4,4]."""
    from . import _lib
    dev = pose.device
    ki = psv_ki_device(tgt_intrinsics, batch, dev).reshape(batch, 9)
    Ks, pose_d = device_cameras(src_intrinsics, pose, batch)
    pose_d = pose_d.reshape(batch, 4, 4)
    ks_b = 0 if Ks.dim() == 2 else Ks.stride(0)
    proj = torch.empty((batch, 16), dtype=_F32, device=dev)
    _lib._call("mpiv_psv_proj_device", Ks, ks_b, pose_d, batch, proj, _lib._stream(dev))
    return ki, proj

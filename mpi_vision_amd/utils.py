"""Drop-in replacement for the hot-path helpers of the reference `utils.py`.

Same function names, argument order, shapes, dtypes and return layouts as
Findeton/mpi-vision `utils.py` (citations below are `utils.py:line`).  The
per-pixel work of every helper runs in hand-written gfx950 HIP kernels in
`libmpiv.so` (C-ABI declared in `include/mpiv.h`); only the tiny 3x3/4x4
per-plane matrices are set up on the host, in torch-CPU fp32 with the
reference's own association order, because their bits decide the 1e-5 parity
(SURVEY.md §8a).

There is no CPU fallback: calling a compute helper without a ROCm device or
without the built library raises.
"""
from __future__ import annotations

import torch

from . import _host, _lib
from .camera import (deprocess_image_torch, make_intrinsics_matrix, parse_camera_lines,  # noqa: F401
                     preprocess_image_torch, read_file_lines, scale_intrinsics)

# The reference keeps a module-level device (utils.py:5).  Every helper reads it
# at call time, exactly like the reference does.
device = torch.device("cuda")


# ---------------------------------------------------------------------------
# Host-only helpers (pure Python / tiny matrices)
# ---------------------------------------------------------------------------

def inv_depths(start_depth, end_depth, num_depths):
    """Plane depths uniform in inverse depth, far->near (utils.py:297-318).

    Reproduces the reference's arithmetic exactly (same expression order), its
    quirk that num_depths < 2 still yields both end points, and its
    descending order."""
    inv_near = 1.0 / start_depth
    inv_far = 1.0 / end_depth
    out = [start_depth, end_depth]
    n_minus_1 = float(num_depths - 1)
    out.extend(1.0 / (inv_near + (inv_far - inv_near) * (float(i) / n_minus_1))
               for i in range(1, num_depths - 1))
    out.sort(reverse=True)
    return out


def meshgrid_abs_torch(batch, height, width):
    """[batch, 3, height, width] grid of (x, y, 1) (utils.py:18-33)."""
    xs = torch.arange(width, dtype=torch.float32).expand(height, width)
    ys = torch.arange(height, dtype=torch.float32).unsqueeze(1).expand(height, width)
    grid = torch.stack([xs, ys, torch.ones(height, width)], 0)
    return grid.unsqueeze(0).repeat(batch, 1, 1, 1).to(device)


def divide_safe_torch(num, den, name=None):
    """num / den with den == 0 replaced by 1e-8 (utils.py:35-39)."""
    return _host.divide_safe(num, den)


def transpose_torch(rot):
    """Swap the last two axes (utils.py:41-42)."""
    return rot.transpose(-2, -1)


def inv_homography_torch(k_s, k_t, rot, t, n_hat, a):
    """Plane-induced target->source homography K_s (R^T + R^T t n R^T / (a - n R^T t)) K_t^-1
    (utils.py:44-67).  Tiny [...,3,3] math, evaluated on the host in torch-CPU fp32
    in the reference's op order (materialised operands, like the reference's
    repeats), and returned on the inputs' device."""
    dev = k_s.device
    host = [_host._cpu32(x).contiguous() for x in (k_s, k_t, rot, t, n_hat, a)]
    return _host.inv_homography(*host).to(dev)


# ---------------------------------------------------------------------------
# Device helpers (HIP kernels)
# ---------------------------------------------------------------------------

def transform_points_torch(points, homography):
    """points [..., H, W, 3] @ homography^T (utils.py:69-88), on the GPU."""
    return _lib.transform_points(points, homography)


def normalize_homogeneous_torch(points):
    """uv / w with w == 0 -> 1e-8 (utils.py:90-101), on the GPU."""
    return _lib.normalize_homogeneous(points)


def bilinear_wrapper_torch(imgs, coords):
    """grid_sample(bilinear, zeros, align_corners=False) of imgs [..., H_s, W_s, C] at
    coords [..., H_t, W_t, 2] in [0,1] (x first).  Returns [..., C, H_t, W_t] like the
    reference (utils.py:104-134)."""
    return _lib.bilinear_sample(imgs, coords, channels_last_out=False)


def resampler_wrapper_torch(imgs, coords):
    """grid_sample of NHWC imgs at coords [N, H', W', 2] -> [N, H', W', C] (utils.py:395-407)."""
    return _lib.bilinear_sample(imgs, coords, channels_last_out=True)


def over_composite(rgbas):
    """Back-to-front over-compositing of a list of [B,H,W,4] images; the first image's
    alpha is ignored (utils.py:136-157)."""
    return _lib.over_composite(rgbas)


def transform_plane_imgs_torch(imgs, pixel_coords_trg, k_s, k_t, rot, t, n_hat, a):
    """Warp [..., H_s, W_s, C] plane images with per-plane homographies; returns
    [..., C, H_t, W_t] (utils.py:160-195, including its x/(H-1), y/(W-1) normalisation)."""
    hom = inv_homography_torch(k_s, k_t, rot, t, n_hat, a)
    return _lib.warp_planes(imgs, pixel_coords_trg, hom)


def planar_transform_torch(imgs, pixel_coords_trg, k_s, k_t, rot, t, n_hat, a):
    """Layer-batched planar transform (utils.py:198-233): imgs [L, B, H, W, C],
    per-batch cameras, per-layer planes -> [L, B, C, H_t, W_t]."""
    n_layers = imgs.shape[0]

    def rep(x):
        return x.unsqueeze(0).repeat((n_layers,) + (1,) * x.dim())

    return transform_plane_imgs_torch(imgs, rep(pixel_coords_trg), rep(k_s), rep(k_t),
                                      rep(rot), rep(t), n_hat, a)


def projective_forward_homography_torch(src_images, intrinsics, pose, depths):
    """Forward-warp [L, B, H, W, C] layers to the target pose (utils.py:237-265);
    returns [L, B, C, H, W]."""
    n_layers, n_batch, height, width, _ = src_images.shape
    rot, t = pose[:, :3, :3], pose[:, :3, 3:]
    n_hat = torch.tensor([0.0, 0.0, 1.0], device=pose.device).reshape(1, 1, 1, 3)
    n_hat = n_hat.repeat(n_layers, n_batch, 1, 1)
    a = -depths.reshape(n_layers, n_batch, 1, 1)
    grid = meshgrid_abs_torch(n_batch, height, width).permute(0, 2, 3, 1)
    return planar_transform_torch(src_images, grid, intrinsics, intrinsics, rot, t, n_hat, a)


def mpi_render_view_torch(rgba_layers, tgt_pose, planes, intrinsics):
    """Render [B, H, W, 3] target views from an MPI [B, H, W, P, 4] (utils.py:267-294).

    `planes` must be a tensor of P depths, far->near (a list raises AttributeError,
    as in the reference, utils.py:279).  The whole warp + over-composite runs as ONE
    fused HIP kernel; the MPI may be a stride-0 broadcast over the batch.  When
    rgba_layers requires grad the result is differentiable w.r.t. it (HIP backward,
    bit-exact to the reference's autograd)."""
    batch_size = tgt_pose.shape[0]
    n_planes = len(planes)
    depths = planes.reshape([n_planes, 1])  # AttributeError on a list, like the reference
    if tgt_pose.is_cuda and rgba_layers.is_cuda:  # poses in HBM: the chain runs there too
        homs = _host.render_homographies_device(tgt_pose, depths.reshape(-1), intrinsics, batch_size)
    else:
        homs = _host.render_homographies(tgt_pose, depths.reshape(-1), intrinsics, batch_size,
                                         pin=rgba_layers.is_cuda)
    if torch.is_grad_enabled() and rgba_layers.requires_grad:
        # training (ipynb cell 12): the adjoint runs in HIP too, bit-exact to the
        # reference's autograd (render_bwd.hip)
        return _lib.RenderFunction.apply(rgba_layers, homs)
    return _lib.render(rgba_layers, homs)


def mpi_render_view_u8(rgba_layers_u8, tgt_pose, planes, intrinsics):
    """mpi_render_view_torch for an 8-bit MPI [B, H, W, P, 4] uint8 (the reference's own
    test-MPI format, test/rgba_*.png): returns exactly
    mpi_render_view_torch(rgba_layers_u8.float() / 255.0, tgt_pose, planes, intrinsics)
    (the reference's image convention, utils.py:324-331) without the float copy: each
    view is packed at 4 B per texel and rendered by render_u8.hip, which converts every
    tap to RN(u8/255) exactly before the reference's blend.  Inference only (no autograd:
    uint8 tensors carry no gradient).  An extension of the drop-in API."""
    batch_size = tgt_pose.shape[0]
    n_planes = len(planes)
    depths = planes.reshape([n_planes, 1])
    if tgt_pose.is_cuda:
        homs = _host.render_homographies_device(tgt_pose, depths.reshape(-1), intrinsics, batch_size)
    else:
        homs = _host.render_homographies(tgt_pose, depths.reshape(-1), intrinsics, batch_size)
    B, H, W, P, _ = rgba_layers_u8.shape
    if B != batch_size or P != n_planes:
        raise RuntimeError(f"shape mismatch: MPI batch/planes {B}/{P} vs poses/planes {batch_size}/{n_planes}")
    homs = homs.reshape(B, P, 9)
    if B > 1 and rgba_layers_u8.stride(0) == 0:  # one MPI, many views: pack once
        return _lib.render_packed_u8(_lib.pack_planes_u8(rgba_layers_u8[0]), homs)
    out = torch.empty((B, H, W, 3), device=rgba_layers_u8.device, dtype=torch.float32)
    packed = None
    for b in range(B):
        packed = _lib.pack_planes_u8(rgba_layers_u8[b], out=packed)
        _lib.render_packed_u8(packed, homs[b:b + 1], out=out[b:b + 1])
    return out


def mpi_from_net_output(mpi_pred, dep):
    """The notebook's MPI assembly (fast-torch-stereo-vision.ipynb cell 10 L79-111):
    the network output [B, 2P+3, H, W] (P blend weights, P alphas, background rgb) and
    dep['ref_img'] [B, H, W, 3] -> rgba_layers [B, H, W, P, 4], P = dep['mpi_planes'].shape[1].
    One HIP pass (assemble.hip) instead of the notebook's P-step torch.cat loop, bit-exact;
    differentiable w.r.t. mpi_pred (HIP backward) when it requires grad."""
    num_mpi_planes = dep['mpi_planes'].shape[1]
    fg_rgb = dep['ref_img'].to(mpi_pred.device)
    if torch.is_grad_enabled() and (mpi_pred.requires_grad or fg_rgb.requires_grad):
        return _lib.AssembleFunction.apply(mpi_pred, fg_rgb, num_mpi_planes)
    return _lib.assemble_mpi(mpi_pred, fg_rgb, num_mpi_planes)


def mpi_render_net_output_torch(mpi_pred, ref_img, tgt_pose, planes, intrinsics):
    """mpi_render_view_torch(mpi_from_net_output(mpi_pred, {'ref_img': ref_img, ...}), tgt_pose,
    planes, intrinsics) -- the two lines of both of the notebook's losses (ipynb cell 12 L7-11,
    L38-42) -- in ONE kernel: each plane's tile footprint is assembled from the network output
    straight into LDS and sampled there (assemble.hip render_netout_kernel); no [B, H, W, P, 4]
    tensor and no packed MPI is written.  Bit-identical to the two-step form.  Differentiable
    w.r.t. mpi_pred and ref_img when either requires grad (_lib.NetOutputRenderFunction: the
    training forward also writes the composite checkpoints; the backward re-assembles the MPI
    for the adjoint, so the MPI is never held between forward and backward), bit-exact to the
    reference's autograd of the two-step form."""
    batch_size = tgt_pose.shape[0]
    n_planes = len(planes)
    depths = planes.reshape([n_planes, 1])
    if tgt_pose.is_cuda:
        homs = _host.render_homographies_device(tgt_pose, depths.reshape(-1), intrinsics, batch_size)
    else:
        homs = _host.render_homographies(tgt_pose, depths.reshape(-1), intrinsics, batch_size)
    fg = ref_img.to(mpi_pred.device)
    if torch.is_grad_enabled() and (mpi_pred.requires_grad or fg.requires_grad):
        return _lib.NetOutputRenderFunction.apply(mpi_pred, fg, homs, n_planes)
    return _lib.render_net_output(mpi_pred, fg, n_planes, homs)


def pixel2cam_torch(depth, pixel_coords, intrinsics, is_homogeneous=True):
    """Back-project pixels to camera space (utils.py:356-375)."""
    return _lib.pixel2cam(depth, pixel_coords, intrinsics, is_homogeneous)


def cam2pixel_torch(cam_coords, proj):
    """Project camera points to pixels [B, H, W, 2] (utils.py:377-393)."""
    return _lib.cam2pixel(cam_coords, proj)


def projective_inverse_warp_torch(img, depth, pose, intrinsics, ret_flows=False):
    """Inverse-warp a source image to the target plane at per-pixel depth
    (utils.py:409-450).  ret_flows=True is broken in the reference (shape mismatch,
    utils.py:447-448) and raises here too."""
    if ret_flows:
        raise RuntimeError("projective_inverse_warp_torch: ret_flows=True is not supported "
                           "(the reference raises a shape mismatch, utils.py:447-448)")
    batch, height, width, _ = img.shape
    ki, proj = _warp_matrices(img, pose, intrinsics, intrinsics)
    return _lib.inverse_warp_depthmap(img, depth, ki, proj, height, width)


def plane_sweep_torch(img, depth_planes, pose, intrinsics):
    """Plane-sweep volume [B, H, W, D*C] (channel d*C+c) of img [B, H, W, C] at the
    listed depths (utils.py:452-471).  One HIP launch writes the whole volume."""
    batch, height, width, _ = img.shape
    return _plane_sweep(img, depth_planes, pose, intrinsics, intrinsics, height, width)


def _plane_sweep(img, depth_planes, pose, src_intrinsics, tgt_intrinsics, height, width, B=None):
    """B given (the unbatched _one calls): img [Hs,Ws,C] and pose [4,4] stand for a batch of 1."""
    if img.is_cuda and pose.is_cuda:  # pose in HBM: proj is formed there, in the sweep's own call
        dev = pose.device
        if B is None:
            B = pose.shape[0]
        stream = torch.cuda.current_stream(dev)
        Ks, pose_d = _host.device_cameras(src_intrinsics, pose, B)
        ki = _host.psv_ki_device(tgt_intrinsics, B, dev, stream.cuda_stream)
        return _lib.plane_sweep_pose(img, depth_planes, ki, Ks, pose_d, height, width, stream)
    if B is not None:
        img, pose = img.unsqueeze(0), pose.unsqueeze(0)
    ki, proj = _host.psv_matrices(_batched(src_intrinsics), _batched(tgt_intrinsics), pose, pin=img.is_cuda)
    return _lib.plane_sweep(img, depth_planes, ki, proj, height, width)


def _batched(k):
    return k.unsqueeze(0) if k.dim() == 2 else k


def _warp_matrices(img, pose, src_intrinsics, tgt_intrinsics):
    if img.is_cuda and pose.is_cuda:
        return _host.psv_matrices_device(src_intrinsics, tgt_intrinsics, pose, pose.shape[0])
    return _host.psv_matrices(src_intrinsics, tgt_intrinsics, pose)


def format_network_input_torch(self, ref_image, psv_src_images, ref_pose, psv_src_poses, planes, intrinsics):
    """Network input [B, H, W, 3 + S*D*3]: the reference image followed by one plane-sweep
    volume per extra source (utils.py:473-498; the unused leading `self` is kept).
    Each source's volume is swept straight into its channel slice of the output
    (no per-source tensors, no torch.cat)."""
    S = psv_src_poses.shape[1]
    inv_ref = torch.inverse(_host._cpu32(ref_pose))
    rel = [torch.matmul(_host._cpu32(psv_src_poses[:, i]), inv_ref) for i in range(S)]  # utils.py:493
    return _lib.network_input(ref_image, psv_src_images, rel, planes, intrinsics)


def plane_sweep_torch_one(img, depth_planes, pose, intrinsics):
    """Unbatched PSV of img [H, W, C]; returns [1, H, W, D*C] (utils.py:513-533).  The
    caller's own intrinsics tensor (not a per-call view of it) keys the memoised inverse."""
    return _plane_sweep(img, depth_planes, pose, intrinsics, intrinsics, img.shape[0], img.shape[1], B=1)


def projective_inverse_warp_torch2(img, depth, pose, src_intrinsics, tgt_intrinsics,
                                   tgt_height, tgt_width, ret_flows=False):
    """Inverse warp with separate source/target intrinsics and target size
    (utils.py:725-769)."""
    if ret_flows:
        raise RuntimeError("projective_inverse_warp_torch2: ret_flows=True is not supported "
                           "(the reference raises a shape mismatch, utils.py:766-767)")
    ki, proj = _warp_matrices(img, pose, src_intrinsics, tgt_intrinsics)
    return _lib.inverse_warp_depthmap(img, depth, ki, proj, tgt_height, tgt_width)


def plane_sweep_torch_one2(img, depth_planes, pose, src_intrinsics, tgt_intrinsics,
                           tgt_height, tgt_width):
    """PSV of img [H_s, W_s, C] into a (tgt_height, tgt_width) target grid with separate
    intrinsics; returns [1, tgt_height, tgt_width, D*C] (utils.py:771-799)."""
    return _plane_sweep(img, depth_planes, pose, src_intrinsics, tgt_intrinsics, tgt_height, tgt_width, B=1)

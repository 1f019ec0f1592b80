"""GPU parity of the low-level helpers (sampler wrappers, over_composite, geometry)
against the reference goldens, bit-exact."""
import numpy as np
import pytest
import torch

from conftest import assert_bits, render_case_inputs

pytestmark = pytest.mark.gpu

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, configs  # noqa: E402


def _t(small, key, dev):
    return torch.tensor(small[key]).to(dev)


def test_bilinear_wrapper(small, dev):
    out = mv.bilinear_wrapper_torch(_t(small, "bil_imgs", dev), _t(small, "bil_coords", dev))
    assert_bits(out.cpu().numpy(), small["bil_out"])


def test_resampler_wrapper(small, dev):
    out = mv.resampler_wrapper_torch(_t(small, "res_imgs", dev), _t(small, "res_coords", dev))
    assert_bits(out.cpu().numpy(), small["res_out"])


def test_over_composite_list(small, dev):
    layers = [t for t in _t(small, "over_in", dev)]
    assert_bits(mv.over_composite(layers).cpu().numpy(), small["over_out"])


def test_over_composite_strided_layers(small, dev):
    """Layers that are views of one permuted tensor (as mpi_render_view_torch makes)."""
    stack = _t(small, "over_in", dev)                     # [P,B,H,W,4]
    perm = stack.permute(1, 2, 3, 0, 4).contiguous()      # [B,H,W,P,4]
    layers = [perm[:, :, :, i] for i in range(stack.shape[0])]
    assert_bits(mv.over_composite(layers).cpu().numpy(), small["over_out"])
    mixed = [layers[0].contiguous()] + layers[1:]
    assert_bits(mv.over_composite(mixed).cpu().numpy(), small["over_out"])


def test_transform_points(small, dev):
    out = mv.transform_points_torch(_t(small, "tp_pts", dev), _t(small, "tp_H", dev))
    assert_bits(out.cpu().numpy(), small["tp_out"])


def test_normalize_homogeneous_mutates_w_like_reference(small, dev):
    pts = _t(small, "nh_in", dev)
    out = mv.normalize_homogeneous_torch(pts)
    assert_bits(out.cpu().numpy(), small["nh_out"])
    assert_bits(pts.cpu().numpy(), small["nh_in_after"])


def test_pixel2cam_cam2pixel(small, dev):
    depth = _t(small, "p2c_depth", dev)
    pix = mv.meshgrid_abs_torch(2, 6, 7)
    cam = mv.pixel2cam_torch(depth, pix, _t(small, "p2c_K", dev))
    assert_bits(cam.cpu().numpy(), small["p2c_out"])
    c2p = mv.cam2pixel_torch(cam, _t(small, "c2p_proj", dev))
    assert_bits(c2p.cpu().numpy(), small["c2p_out"])


def test_layer_pipeline_helpers_match_render(small, meta, dev):
    """projective_forward_homography_torch + over_composite of its planes ==
    the fused render, i.e. the unfused helper chain of the reference (utils.py:283-293)."""
    mpi = render_case_inputs(meta["small"], "render_a").to(dev)
    pose, K, planes = _t(small, "render_a_pose", dev), _t(small, "render_a_K", dev), _t(small, "render_a_depths", dev)
    layers = mpi.permute(3, 0, 1, 2, 4)
    depths = planes.reshape(-1, 1).repeat(1, 2)
    proj = mv.projective_forward_homography_torch(layers, K, pose, depths)   # [P,B,4,H,W]
    proj = proj.permute(0, 1, 3, 4, 2)
    out = mv.over_composite([proj[i] for i in range(proj.shape[0])])
    assert_bits(out.cpu().numpy(), small["render_a_out"])


def test_meshgrid(dev):
    g = mv.meshgrid_abs_torch(2, 3, 4).cpu()
    assert g.shape == (2, 3, 3, 4)
    assert torch.equal(g[1, 0, 2], torch.arange(4.0)) and torch.equal(g[0, 1, :, 1], torch.arange(3.0))
    assert torch.all(g[:, 2] == 1)


def test_device_homographies_bit_exact(dev):
    """mpiv_render_homographies_device (the chain on the GPU, used when poses live in HBM)
    equals the host chain bit for bit: random rotations / translations, a pose whose
    den == 0 branch fires, several batch sizes; and the K^-1 memo follows in-place edits."""
    from mpi_vision_amd import configs
    from mpi_vision_amd import _host
    g = torch.Generator().manual_seed(17)
    for B, P in ((1, 10), (7, 33), (64, 128)):
        poses = []
        for k in range(B):
            t = ((torch.rand(3, generator=g) - 0.5) * (0.3 + k)).tolist()
            poses.append(configs.pose_from(configs.rot_y(float(torch.rand(1, generator=g)) * 40 - 20), t))
        if B > 1:
            poses[1] = configs.pose_from(configs.rot_y(0.0), (0.0, 0.0, 2.0))  # a - c == 0 at depth 2
        pose = configs.f32(poses)
        depths = configs.f32(configs.inv_depths(1, 100, P) if B != 7 else [2.0] + configs.inv_depths(1, 100, P - 1))
        K = configs.f32([configs.intrinsics_matrix(500.0 + k, 480.0, 320.0, 200.0 + k) for k in range(B)])
        want = _host.render_homographies(pose, depths, K, B).numpy()
        Kd = K.to(dev)
        got = _host.render_homographies_device(pose.to(dev), depths.to(dev), Kd, B)
        assert_bits(got.cpu().numpy(), want, f"B={B}")
        Kd.mul_(1.5)  # in place: the memoised inverse must not be reused
        want2 = _host.render_homographies(pose, depths, K * 1.5, B).numpy()
        got2 = _host.render_homographies_device(pose.to(dev), depths.to(dev), Kd, B)
        assert_bits(got2.cpu().numpy(), want2, f"B={B} after in-place K update")


def test_device_psv_matrices_bit_exact(dev):
    """psv_matrices_device (Ki memoised per intrinsics tensor, proj = K4 @ pose by
    mpiv_psv_proj_device) equals the host psv_matrices bit for bit, for one camera [3,3]
    shared by the batch and for per-view [B,3,3] intrinsics, and again after an in-place
    update of K (the memo follows the tensor's version)."""
    g = torch.Generator().manual_seed(4)
    c = configs.config4()
    B = 40
    pose = configs.f32(c["poses"][200:200 + B])
    K = configs.f32([configs.intrinsics_matrix(*(torch.rand(4, generator=g) * 300 + 5).tolist()) for _ in range(B)])
    Kd, posed = K.to(dev), pose.to(dev)
    for _ in range(2):
        ki, proj = _host.psv_matrices_device(Kd, Kd, posed, B)
        wki, wproj = _host.psv_matrices(K, K, pose)
        assert_bits(ki.cpu().numpy(), wki.numpy())
        assert_bits(proj.cpu().numpy(), wproj.numpy())
    K1 = Kd[7].clone()
    for scale in (1.0, 1.5):
        K1.mul_(scale)
        # one camera for the batch, passed the way the reference's caller would: expanded
        # (stride 0).  The reference inverts that tensor as laid out (utils.py:370), and so must
        # both drop-in paths (tests/test_kstride.py holds the reference goldens for it)
        Ke = K1[None].expand(B, 3, 3)
        ki, proj = _host.psv_matrices_device(Ke, Ke, posed, B)
        Kh = K1.cpu()[None].expand(B, 3, 3)
        wki, wproj = _host.psv_matrices(Kh, Kh, pose)
        assert_bits(ki.cpu().numpy(), wki.numpy())
        assert_bits(ki.cpu().numpy(), torch.inverse(Kh).reshape(B, 9).numpy())
        assert_bits(proj.cpu().numpy(), wproj.numpy())
        # an unbatched [3,3] camera: inverted once as given, broadcast over the batch
        ki, proj = _host.psv_matrices_device(K1, K1, posed, B)
        wki, wproj = _host.psv_matrices(K1.cpu(), K1.cpu(), pose)
        assert_bits(ki.cpu().numpy(), wki.numpy())
        assert_bits(proj.cpu().numpy(), wproj.numpy())

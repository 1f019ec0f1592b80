"""CPU: host-side logic of the drop-in -- plane depths, homography / PSV matrix
setup (bit-exact vs the reference's H), API error behaviour, no CPU fallback."""
import numpy as np
import pytest
import torch

from conftest import RENDER_CASES, assert_bits

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, configs  # noqa: E402


@pytest.mark.parametrize("n", [1, 2, 3, 10, 32, 64, 128, 256])
def test_inv_depths_exact(n, small):
    got = np.array(mv.inv_depths(1, 100, n), dtype=np.float64)
    assert np.array_equal(got, small[f"inv_depths_{n}"])


def test_inv_depths_other_range(small):
    assert np.array_equal(np.array(mv.inv_depths(0.5, 20.0, 7)), small["inv_depths_0.5_20_7"])


@pytest.mark.parametrize("name", RENDER_CASES)
def test_render_homographies_bit_exact(name, small):
    B = small[f"{name}_pose"].shape[0]
    H = _host.render_homographies(torch.tensor(small[f"{name}_pose"]), torch.tensor(small[f"{name}_depths"]),
                                  torch.tensor(small[f"{name}_K"]), B)
    P = small[f"{name}_depths"].shape[0]
    assert_bits(H.numpy(), small[f"{name}_H"].transpose(1, 0, 2, 3).reshape(B, P, 9), name)


@pytest.mark.parametrize("name", RENDER_CASES)
def test_native_homography_chain_equals_torch_ops(name, small):
    """The library's host restatement of the chain (mpiv_render_homographies) equals the
    op-by-op torch form on the same inputs, and both equal the reference's H."""
    B = small[f"{name}_pose"].shape[0]
    args = (torch.tensor(small[f"{name}_pose"]), torch.tensor(small[f"{name}_depths"]),
            torch.tensor(small[f"{name}_K"]), B)
    assert_bits(_host.render_homographies(*args).numpy(), _host.render_homographies_torch(*args).numpy(), name)


def test_native_homography_chain_random_poses():
    """Random poses / intrinsics / depths (incl. a plane through the camera centre, where
    divide_safe's den == 0 branch fires): native chain == torch ops, bit for bit."""
    g = torch.Generator().manual_seed(99)
    B, P = 6, 40
    poses = []
    for k in range(B):
        R = configs.rot_y(float(torch.rand(1, generator=g)) * 40 - 20)
        poses.append(configs.pose_from(R, ((torch.rand(3, generator=g) - 0.5) * 3).tolist()))
    poses[0] = configs.pose_from(configs.rot_y(0.0), (0.3, -0.2, -7.5))  # n R^T t = t_z exactly
    pose = configs.f32(poses)
    K = configs.f32([configs.intrinsics_matrix(*(torch.rand(4, generator=g) * 200 + 10).tolist()) for _ in range(B)])
    d = (torch.rand(P, generator=g) * 50 + 0.1).sort(descending=True).values
    d[5] = 7.5  # a - n R^T t = -7.5 - (-7.5) == 0 for view 0: the 1e-8 branch
    H = _host.render_homographies_torch(pose, d, K, B)
    assert torch.isfinite(H).all() and H.abs().max() > 1e6  # the branch fired (division by 1e-8)
    assert_bits(_host.render_homographies(pose, d, K, B).numpy(), _host.render_homographies_torch(pose, d, K, B).numpy())


def test_inv_homography_helper_bit_exact(small):
    K, pose, d = (torch.tensor(small[k]) for k in ("hom_K", "hom_pose", "hom_depths"))
    P, B = d.shape[0], K.shape[0]
    rep = lambda x: x.unsqueeze(0).repeat((P,) + (1,) * x.dim())  # noqa: E731
    n_hat = torch.tensor([0.0, 0.0, 1.0]).reshape(1, 1, 1, 3).repeat(P, B, 1, 1)
    a = -d.reshape(P, 1).repeat(1, B).reshape(P, B, 1, 1)
    H = mv.inv_homography_torch(rep(K), rep(K), rep(pose[:, :3, :3]), rep(pose[:, :3, 3:]), n_hat, a)
    assert_bits(H.numpy(), small["hom_H"])
    # expanded (stride-0) operands are materialised like the reference's repeats
    exp = lambda x: x.unsqueeze(0).expand((P,) + tuple(x.shape))  # noqa: E731
    H2 = mv.inv_homography_torch(exp(K), exp(K), exp(pose[:, :3, :3]), exp(pose[:, :3, 3:]), n_hat, a)
    assert_bits(H2.numpy(), small["hom_H"])


def test_c4_homographies_match_reference(large):
    for pose_index in (0, 500):
        H = _host.render_homographies(torch.tensor(large[f"c4_{pose_index}_pose"]), torch.tensor(large["c4_depths"]),
                                      torch.tensor(large["c4_K"]), 1)
        assert_bits(H.numpy(), large[f"c4_{pose_index}_H"].transpose(1, 0, 2, 3).reshape(1, 128, 9))


def test_psv_matrices():
    K = configs.f32([configs.intrinsics_matrix(100.0, 110.0, 30.0, 20.0)])
    pose = configs.f32([configs.pose_from(configs.rot_y(2.0), (0.1, 0.0, 0.2))])
    ki, proj = _host.psv_matrices(K, K, pose)
    assert torch.equal(ki.reshape(1, 3, 3), torch.inverse(K))
    k4 = torch.eye(4)[None].clone()
    k4[:, :3, :3] = K
    assert torch.equal(proj.reshape(1, 4, 4), torch.matmul(k4, pose))


def test_divide_safe():
    num = torch.tensor([1.0, 2.0, 3.0])
    den = torch.tensor([0.0, -0.0, 4.0])
    out = mv.divide_safe_torch(num, den)
    assert torch.equal(out, num / torch.tensor([1e-8, 1e-8, 4.0]))


def test_meshgrid_values():
    mv.utils.device = torch.device("cpu")
    try:
        g = mv.meshgrid_abs_torch(2, 3, 4)
    finally:
        mv.utils.device = torch.device("cuda")
    assert g.shape == (2, 3, 3, 4)
    assert torch.equal(g[0, 0, 1], torch.arange(4.0)) and torch.equal(g[1, 1, :, 2], torch.arange(3.0))


def test_no_cpu_fallback():
    """The product path refuses CPU tensors instead of silently computing on the host."""
    mpi = torch.zeros((1, 4, 4, 2, 4))
    with pytest.raises(RuntimeError, match="no CPU path"):
        mv.mpi_render_view_torch(mpi, torch.eye(4)[None], torch.tensor([2.0, 1.0]), torch.eye(3)[None])
    with pytest.raises(RuntimeError, match="no CPU path"):
        mv.plane_sweep_torch(torch.zeros((1, 4, 4, 3)), [1.0, 2.0], torch.eye(4)[None], torch.eye(3)[None])
    with pytest.raises(RuntimeError, match="no CPU path"):
        mv.over_composite([torch.zeros((1, 2, 2, 4))] * 2)


def test_planes_must_be_tensor():
    with pytest.raises(AttributeError):  # utils.py:279 behaviour
        mv.mpi_render_view_torch(torch.zeros((1, 4, 4, 2, 4)), torch.eye(4)[None], [2.0, 1.0], torch.eye(3)[None])


def test_ret_flows_unsupported():
    with pytest.raises(RuntimeError):
        mv.projective_inverse_warp_torch(torch.zeros((1, 4, 4, 3)), torch.ones((1, 4, 4)), torch.eye(4)[None],
                                         torch.eye(3)[None], ret_flows=True)


def test_configs():
    c4 = configs.config4()
    assert len(c4["poses"]) == 1000 and len(c4["depths"]) == 128
    assert c4["depths"][0] == 100 and c4["depths"][-1] == 1
    c1 = configs.config1_camera()
    assert abs(c1["K"][0][0] - 554.2562584220408) < 1e-9


def test_plane_sweep_no_depths_raises_value_error():
    """No depth planes: the reference's torch.cat raises ValueError (utils.py:470); the
    drop-in raises it before touching a device (so also for a CPU tensor)."""
    import mpi_vision_amd as mv
    K = torch.tensor([[[40.0, 0, 26], [0, 41.0, 14], [0, 0, 1]]])
    with pytest.raises(ValueError, match="non-empty list"):
        mv.plane_sweep_torch(torch.rand(1, 12, 16, 3), [], torch.eye(4)[None], K)


def _psv_proj_host(Ks, pose):
    from mpi_vision_amd import _lib
    B = pose.shape[0]
    Ks = Ks.contiguous()
    pose = pose.contiguous()
    out = torch.empty((B, 16), dtype=torch.float32)
    ks_b = 0 if Ks.dim() == 2 else 9
    rc = _lib.load().mpiv_psv_proj(Ks.data_ptr(), ks_b, pose.data_ptr(), B, out.data_ptr())
    assert rc == 0
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_psv_proj_restatement_equals_torch(seed):
    """mpiv_psv_proj (geometry.hip psv_proj, the code the device entry runs too) equals
    psv_matrices' torch-CPU proj = cat(K, 0; 0 0 0 1) @ pose bit for bit (utils.py:428-438):
    camera-path poses, random dense 4x4 "poses" with negative zeros and signed entries, and
    intrinsics with and without skew."""
    g = torch.Generator().manual_seed(seed)
    B = 64
    c = configs.config4()
    poses = configs.f32(c["poses"][seed * 100:seed * 100 + B // 2])
    rnd = (torch.rand((B // 2, 4, 4), generator=g) - 0.5) * 10
    rnd[:, 1, 2] = -0.0
    rnd[0] = torch.tensor([[-0.0, 0.0, -1.0, 2.0], [0.0, -0.0, 0.0, -0.0], [1.0, 0.0, -0.0, 0.5], [0.0, -0.0, 0.0, 1.0]])
    pose = torch.cat([poses, rnd])
    K = configs.f32([configs.intrinsics_matrix(*(torch.rand(4, generator=g) * 300 + 5).tolist()) for _ in range(B)])
    K[::3, 0, 1] = torch.rand(K[::3].shape[0], generator=g) - 0.5  # skew
    ki, proj = _host.psv_matrices(K, K, pose)
    assert_bits(_psv_proj_host(K, pose).numpy(), proj.numpy())
    ki1, proj1 = _host.psv_matrices(K[:1].expand(B, 3, 3), K[:1].expand(B, 3, 3), pose)
    assert_bits(_psv_proj_host(K[0], pose).numpy(), proj1.numpy())

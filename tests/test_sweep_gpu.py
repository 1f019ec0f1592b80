"""GPU parity of the plane-sweep / inverse-warp kernels against the reference
goldens (bit-exact)."""
import numpy as np
import pytest
import torch

from conftest import assert_bits, psv_case_input, sha256

pytestmark = pytest.mark.gpu

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import configs  # noqa: E402


def _t(small, key, dev):
    return torch.tensor(small[key]).to(dev)


def test_plane_sweep_batched(small, meta, dev):
    img = psv_case_input(meta["small"], "psv_a")
    out = mv.plane_sweep_torch(img.to(dev), list(small["psv_a_depths"]), _t(small, "psv_a_pose", dev),
                               _t(small, "psv_a_K", dev))
    assert_bits(out.cpu().numpy(), small["psv_a_out"])


def test_plane_sweep_one(small, meta, dev):
    img = psv_case_input(meta["small"], "psv_one")
    out = mv.plane_sweep_torch_one(img.to(dev), list(small["psv_one_depths"]), _t(small, "psv_one_pose", dev),
                                   _t(small, "psv_one_K", dev))
    assert out.shape == small["psv_one_out"].shape
    assert_bits(out.cpu().numpy(), small["psv_one_out"])


def test_plane_sweep_one2_separate_intrinsics(small, meta, dev):
    img = psv_case_input(meta["small"], "psv_two")
    m = meta["small"]["psv_two"]
    out = mv.plane_sweep_torch_one2(img.to(dev), list(small["psv_two_depths"]), _t(small, "psv_two_pose", dev),
                                    _t(small, "psv_two_Ks", dev), _t(small, "psv_two_Kt", dev), m["tgt_h"], m["tgt_w"])
    assert_bits(out.cpu().numpy(), small["psv_two_out"])


def test_plane_sweep_strided_input(small, meta, dev):
    img = psv_case_input(meta["small"], "psv_a")
    wide = torch.zeros((2, 48, 64, 5))
    wide[..., 1:4] = img
    view = wide.to(dev)[..., 1:4]
    out = mv.plane_sweep_torch(view, list(small["psv_a_depths"]), _t(small, "psv_a_pose", dev),
                               _t(small, "psv_a_K", dev))
    assert_bits(out.cpu().numpy(), small["psv_a_out"])


def test_inverse_warp_single_depth(small, meta, dev):
    """projective_inverse_warp_torch at one depth == that depth's slice of the PSV."""
    img = psv_case_input(meta["small"], "psv_a").to(dev)
    d = float(small["psv_a_depths"][2])
    depth = torch.full((2, 48, 64), d, device=dev)
    out = mv.projective_inverse_warp_torch(img, depth, _t(small, "psv_a_pose", dev), _t(small, "psv_a_K", dev))
    assert_bits(out.cpu().numpy(), small["psv_a_out"][..., 6:9])


def test_plane_sweep_c3(large, meta, dev):
    """Config 3: 5 x 1024x768 sources -> 64 planes (the full [5,768,1024,192] volume)."""
    c3 = configs.config3()
    g = torch.Generator().manual_seed(c3["seed"])
    img = torch.rand((c3["S"], c3["H"], c3["W"], 3), generator=g, dtype=torch.float32)
    assert sha256(img) == meta["large"]["c3"]["img_sha"]
    out = mv.plane_sweep_torch(img.to(dev), c3["depths"], _t(large, "c3_pose", dev), _t(large, "c3_K", dev))
    flat = out.reshape(-1)
    idx = torch.from_numpy(large["c3_idx"]).to(dev)
    np.testing.assert_array_equal(flat[idx].cpu().numpy(), large["c3_val"])
    for i in range(c3["S"]):
        assert sha256(out[i]) == meta["large"]["c3"]["per_source_sha"][i]


def test_format_network_input(small, dev):
    """format_network_input_torch (utils.py:473-498): ref image + one PSV per source,
    concatenated on channels; bit-exact."""
    t = {k: torch.tensor(small[f"fni_{k}"]) for k in ("ref", "src", "ref_pose", "src_poses", "K")}
    out = mv.format_network_input_torch(None, t["ref"].to(dev), t["src"].to(dev), t["ref_pose"].to(dev),
                                        t["src_poses"].to(dev), list(small["fni_planes"]), t["K"].to(dev))
    assert_bits(out.cpu().numpy(), small["fni_out"])


@pytest.mark.parametrize("store", [None, "0", "1", "2"])
def test_plane_sweep_store_modes(store, small, meta, dev, monkeypatch):
    """The tile sweep kernel (default) and every output-store path of the grouped
    kernel (scalar, 16-B per lane, LDS-staged dense run; MPIV_SWEEP_STORE selects it)
    give the reference bits, incl. a partial last depth group (D = 6, 5) and C = 4."""
    if store is not None:
        monkeypatch.setenv("MPIV_SWEEP_STORE", store)
    img = psv_case_input(meta["small"], "psv_a")
    out = mv.plane_sweep_torch(img.to(dev), list(small["psv_a_depths"]), _t(small, "psv_a_pose", dev),
                               _t(small, "psv_a_K", dev))
    assert_bits(out.cpu().numpy(), small["psv_a_out"])
    img = psv_case_input(meta["small"], "psv_one")
    out = mv.plane_sweep_torch_one(img.to(dev), list(small["psv_one_depths"]), _t(small, "psv_one_pose", dev),
                                   _t(small, "psv_one_K", dev))
    assert_bits(out.cpu().numpy(), small["psv_one_out"])
    img = psv_case_input(meta["small"], "psv_two")
    m = meta["small"]["psv_two"]
    out = mv.plane_sweep_torch_one2(img.to(dev), list(small["psv_two_depths"]), _t(small, "psv_two_pose", dev),
                                    _t(small, "psv_two_Ks", dev), _t(small, "psv_two_Kt", dev), m["tgt_h"], m["tgt_w"])
    assert_bits(out.cpu().numpy(), small["psv_two_out"])


def test_plane_sweep_many_depths_vs_oracle(dev):
    """D = 150 (three LDS depth chunks, a partial last one), C = 2, odd sizes, two views:
    bit-exact to the oracle."""
    from mpi_vision_amd import _host
    from oracle import oracle
    g = torch.Generator().manual_seed(12)
    B, H, W, C, D = 2, 37, 83, 2, 150
    img = torch.rand((B, H, W, C), generator=g)
    K = configs.f32([configs.intrinsics_matrix(50.0, 52.0, 41.0, 18.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(2.0 * k - 1), (0.1 * k - 0.05, 0.02, 0.01)) for k in range(B)])
    depths = configs.inv_depths(0.7, 60, D)
    out = mv.plane_sweep_torch(img.to(dev), depths, poses.to(dev), K.to(dev))
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, H, W)
    assert_bits(out.cpu().numpy(), want)

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


@pytest.mark.parametrize("rows", [6, 8])
@pytest.mark.parametrize("D", [3, 10, 64])
def test_plane_sweep_tall_tiles_vs_oracle(rows, D, dev, kopts):
    """The depth-per-lane sweep with 6- and 8-row tiles (sweep_rows; 4096-texel staging box):
    partial tiles, off-image footprints and the swapped normalisation, bit-exact vs the oracle."""
    from mpi_vision_amd import _host
    from oracle import oracle
    kopts(sweep_rows=rows)
    g = torch.Generator().manual_seed(D + rows)
    B, H, W = 2, 45, 100
    img = torch.rand((B, H, W, 3), generator=g)
    K = configs.f32([configs.intrinsics_matrix(80.0, 85.0, W / 2.0, H / 2.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(3.0), (0.2, 0.03, 0.0)),
                         configs.pose_from(configs.rot_y(-1.0), (-0.1, 0.0, 0.05))])
    depths = configs.inv_depths(1, 100, D)
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, H, W)
    out = mv.plane_sweep_torch(img.to(dev), depths, poses.to(dev), K.to(dev))
    assert_bits(out.cpu().numpy(), want)


def test_plane_sweep_one_notebook_call_pattern(small, meta, dev):
    """The notebook's dataset call (ipynb cell 8 L73-75): the depths are a DEVICE tensor
    (torch.Tensor(inv_depths(...)).to(device)) and pose / intrinsics live on the device; the
    reference iterates the tensor element by element -- same volume as the depth list.
    Repeated calls (the memoised depth upload, the single pinned matrix upload) stay equal."""
    img = psv_case_input(meta["small"], "psv_one").to(dev)
    planes = torch.Tensor(list(small["psv_one_depths"])).to(dev)
    pose, K = _t(small, "psv_one_pose", dev), _t(small, "psv_one_K", dev)
    for _ in range(3):
        out = mv.plane_sweep_torch_one(img, planes, pose, K)
        assert_bits(out.cpu().numpy(), small["psv_one_out"])
        out = mv.plane_sweep_torch_one(img, list(small["psv_one_depths"]), pose, K)
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


@pytest.mark.parametrize("dlane", ["1", "0"])
def test_plane_sweep_c3(dlane, large, meta, dev, kopts):
    """Config 3: 5 x 1024x768 sources -> 64 planes (the full [5,768,1024,192] volume), through
    the depth-per-lane LDS kernel (default for D % 64 == 0) and the pixel-per-lane one."""
    kopts(sweep_dlane=dlane)
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


@pytest.mark.parametrize("store", [None, "shrink", "padded", "pixlane", "pixlane-shrink", "tile", "0", "1", "2"])
def test_plane_sweep_store_modes(store, small, meta, dev, kopts, monkeypatch):
    """Every sweep kernel through the drop-ins gives the reference bits, incl. a partial last
    depth group (D = 6, 5): the default depth-per-lane kernel on the source in place ("shrink"
    forces its per-sample global fallback) and, on a padded texel copy (the drop-ins routed
    through _lib.plane_sweep_padded), the same kernel, the pixel-per-lane LDS kernel, the tile
    kernel and every output-store path of the grouped kernel (scalar, 16-B per lane,
    LDS-staged dense run; debug option sweep_store)."""
    from mpi_vision_amd import _lib
    if store not in (None, "shrink"):
        monkeypatch.setattr(_lib, "plane_sweep", _lib.plane_sweep_padded)
    if store in ("shrink", "pixlane-shrink"):
        kopts(box_shrink=2)
    if store in ("pixlane", "pixlane-shrink"):
        kopts(sweep_dlane=0)
    elif store == "tile":
        kopts(sweep_tile=1)
    elif store in ("0", "1", "2"):
        kopts(sweep_store=store)
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


@pytest.mark.parametrize("C", [1, 2, 3, 4])
@pytest.mark.parametrize("shrink", ["0", "3"])
@pytest.mark.parametrize("path", ["raw", "padded", "pixlane"])
def test_plane_sweep_lds_vs_oracle(C, shrink, path, dev, kopts):
    """The LDS-staged sweep with C = 1 and 4, a target size whose rows end in a partial
    64-pixel segment, separate source / target intrinsics and sizes (the _one2 geometry):
    bit-exact to the oracle, also with every staged box shrunk (box_shrink: most
    samples take the per-sample global fallback)."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    kopts(box_shrink=shrink, sweep_dlane=0 if path == "pixlane" else 1)
    g = torch.Generator().manual_seed(31 + C)
    B, Hs, Ws, D, Ht, Wt = 2, 45, 97, 11, 38, 131
    img = torch.rand((B, Hs, Ws, C), generator=g)
    Ks = configs.f32([configs.intrinsics_matrix(60.0, 61.0, 48.0, 22.0)] * B)
    Kt = configs.f32([configs.intrinsics_matrix(80.0, 79.0, 65.0, 19.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(3.0 * k - 1.5), (0.2 * k - 0.1, 0.03, -0.02))
                         for k in range(B)])
    depths = configs.inv_depths(0.8, 40, D)
    ki, proj = _host.psv_matrices(Ks, Kt, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Ht, Wt)
    sweep = _lib.plane_sweep if path == "raw" else _lib.plane_sweep_padded
    out = sweep(img.to(dev), depths, ki, proj, Ht, Wt)
    assert_bits(out.cpu().numpy(), want, f"C={C} shrink={shrink} {path}")


@pytest.mark.parametrize("dlane", ["1", "0"])
def test_plane_sweep_more_depths_than_lds_table(dlane, dev, kopts):
    """D = 1030 > the pixel-per-lane kernel's LDS depth table: the depth-per-lane kernel
    (17 chunks, default) or the tile kernel takes over, still bit-exact."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    kopts(sweep_dlane=dlane)
    g = torch.Generator().manual_seed(5)
    img = torch.rand((1, 9, 13, 3), generator=g)
    K = configs.f32([configs.intrinsics_matrix(12.0, 12.5, 6.0, 4.0)])
    pose = configs.f32([configs.pose_from(configs.rot_y(2.0), (0.05, 0.01, 0.0))])
    depths = configs.inv_depths(0.5, 50, 1030)
    ki, proj = _host.psv_matrices(K, K, pose)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, 9, 13)
    sweep = _lib.plane_sweep if dlane == "1" else _lib.plane_sweep_padded
    assert_bits(sweep(img.to(dev), depths, ki, proj, 9, 13).cpu().numpy(), want)


@pytest.mark.parametrize("C", [3, 4])
def test_plane_sweep_off_image_tiles(C, dev):
    """Landscape sources (the swapped x / H normalisation pushes every sample past x = 3W/4
    off the image), a strong sideways baseline and a source looking away: many tiles have
    footprints wholly off the image (zero-tile stores and border-collapsed boxes), others
    straddle the edge; bit-exact to the oracle, output zeros included (+0.0)."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    g = torch.Generator().manual_seed(77 + C)
    B, Hs, Ws, D = 3, 60, 160, 16
    img = torch.rand((B, Hs, Ws, C), generator=g) + 0.5
    K = configs.f32([configs.intrinsics_matrix(150.0, 150.0, 80.0, 30.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(0.5), (0.1, 0.01, 0.0)),
                         configs.pose_from(configs.rot_y(-20.0), (1.5, 0.2, 0.1)),
                         configs.pose_from(configs.rot_y(40.0), (-2.0, -0.5, 0.3))])
    depths = configs.inv_depths(1, 50, D)
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Hs, Ws)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Hs, Ws)
    got = out.cpu().numpy()
    assert_bits(got, want, f"C={C}")
    assert (want == 0).mean() > 0.2  # the case does exercise off-image samples


@pytest.mark.parametrize("C", [5, 7])
def test_plane_sweep_wide_channels_vs_oracle(C, dev):
    """C > 4 (the reference sweeps any channel count, e.g. stacked sources): the generic
    strided kernel, bit-exact to the oracle, through the plane_sweep_torch drop-in."""
    from mpi_vision_amd import _host
    from oracle import oracle
    g = torch.Generator().manual_seed(70 + C)
    B, H, W, D = 2, 29, 53, 6
    img = torch.rand((B, H, W, C), generator=g)
    K = configs.f32([configs.intrinsics_matrix(40.0, 41.0, 26.0, 14.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(2.0 * k - 1.0), (0.1 * k - 0.05, 0.02, 0.0))
                         for k in range(B)])
    depths = configs.inv_depths(1.0, 30, D)
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, H, W)
    out = mv.plane_sweep_torch(img.to(dev), depths, poses.to(dev), K.to(dev))
    assert out.shape == (B, H, W, D * C)
    assert_bits(out.cpu().numpy(), want, f"C={C}")


def test_plane_sweep_empty_inputs_raise_like_reference(dev):
    """The reference raises on every empty input (measured: ValueError from torch.cat for
    no depths, RuntimeError from its reshapes for an empty batch or image); so does the
    drop-in, before any launch."""
    K = configs.f32([configs.intrinsics_matrix(40.0, 41.0, 26.0, 14.0)])
    pose = configs.f32([configs.pose_from(configs.rot_y(1.0), (0.05, 0.0, 0.0))])
    img = torch.rand((1, 12, 16, 3), device=dev)
    with pytest.raises(ValueError, match="non-empty list"):
        mv.plane_sweep_torch(img, [], pose.to(dev), K.to(dev))
    with pytest.raises(RuntimeError):
        mv.plane_sweep_torch(img[:0], [1.0, 2.0], pose[:0].to(dev), K[:0].to(dev))
    with pytest.raises(RuntimeError):
        mv.plane_sweep_torch(img[:, :0], [1.0, 2.0], pose.to(dev), K.to(dev))


@pytest.mark.parametrize("C", [1, 2, 3, 4])
@pytest.mark.parametrize("dlane", ["0", "1"])
def test_plane_sweep_pixel_interleaved_store_all_channels(C, dlane, dev, kopts):
    """Whole 16-pixel blocks and whole sets of 4 depth groups (Wt % 64 == 0, D % 16 == 0):
    the LDS kernel's pixel-interleaved order and its swizzled per-wave store slot (a
    different row rotation for C = 3 than for C = 1, 2, 4), bit-exact to the oracle."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    kopts(sweep_dlane=dlane)  # 0: the pixel-per-lane kernel's pixel-interleaved store path (padded input)
    g = torch.Generator().manual_seed(90 + C)
    B, Hs, Ws, D, Ht, Wt = 2, 40, 96, 32, 12, 128
    img = torch.rand((B, Hs, Ws, C), generator=g)
    Ks = configs.f32([configs.intrinsics_matrix(60.0, 61.0, 48.0, 20.0)] * B)
    Kt = configs.f32([configs.intrinsics_matrix(80.0, 79.0, 64.0, 6.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(2.0 * k - 1.0), (0.1 * k - 0.05, 0.02, 0.0))
                         for k in range(B)])
    depths = configs.inv_depths(1.0, 40, D)
    ki, proj = _host.psv_matrices(Ks, Kt, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Ht, Wt)
    out = (_lib.plane_sweep_padded if dlane == "0" else _lib.plane_sweep)(img.to(dev), depths, ki, proj, Ht, Wt)
    assert_bits(out.cpu().numpy(), want, f"C={C}")


@pytest.fixture(scope="module")
def warp():
    import os
    from conftest import GOLD
    return np.load(os.path.join(GOLD, "warp.npz"))


@pytest.mark.parametrize("c", ["piw", "piw4"])
def test_inverse_warp_depth_map_vs_reference(warp, dev, c):
    """projective_inverse_warp_torch (utils.py:409-450) with NON-constant depth maps --
    depth 0, negative depths, near/far mixes, 3 and 4 channels -- bit-exact to the
    reference (tests/golden/warp.npz, tools/gen_goldens_warp.py)."""
    t = {k: torch.tensor(warp[f"{c}_{k}"]).to(dev) for k in ("img", "depth", "pose", "K")}
    out = mv.projective_inverse_warp_torch(t["img"], t["depth"], t["pose"], t["K"])
    assert_bits(out, warp[f"{c}_out"], c)
    # a strided (non-contiguous) depth map and image read in place give the same bits
    wide_d = torch.zeros(t["depth"].shape[:2] + (t["depth"].shape[2] + 3,), device=dev)
    wide_d[..., 1:-2] = t["depth"]
    wide_i = torch.zeros(t["img"].shape[:3] + (t["img"].shape[3] + 2,), device=dev)
    wide_i[..., 1:-1] = t["img"]
    out_s = mv.projective_inverse_warp_torch(wide_i[..., 1:-1], wide_d[..., 1:-2], t["pose"], t["K"])
    assert_bits(out_s, warp[f"{c}_out"], c + " strided")


def test_inverse_warp2_depth_map_vs_reference(warp, dev):
    """projective_inverse_warp_torch2 (utils.py:725-769): separate source / target
    intrinsics, a 28x70 target grid from a 36x48 source, a random depth map: bit-exact."""
    t = {k: torch.tensor(warp[f"piw2_{k}"]).to(dev) for k in ("img", "depth", "pose", "Ks", "Kt")}
    Ht, Wt = (int(v) for v in warp["piw2_tgt"])
    out = mv.projective_inverse_warp_torch2(t["img"], t["depth"], t["pose"], t["Ks"], t["Kt"], Ht, Wt)
    assert_bits(out, warp["piw2_out"], "piw2")


@pytest.mark.parametrize("band", [1, 0])
@pytest.mark.parametrize("C", [1, 2, 3, 4])
@pytest.mark.parametrize("D", [6, 10, 16, 64, 100, 128])
@pytest.mark.parametrize("shrink", ["0", "3"])
def test_plane_sweep_depth_lanes_vs_oracle(C, D, shrink, band, dev, kopts):
    """The depth-per-lane LDS kernel: D <= 64 (64 // D pixels per wave slot, idle lanes when
    D does not divide 64), D > 64 (64-depth chunks, a partial last one); odd target sizes (a
    partial last 64-pixel segment and 4-row tile), separate source / target intrinsics; also
    with shrunk boxes (most samples through its global fallback): bit-exact to the oracle."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    kopts(box_shrink=shrink, sweep_band=band)  # band 1: the band-walking ring kernel (round 5 default)
    g = torch.Generator().manual_seed(140 + C + D)
    B, Hs, Ws, Ht, Wt = 2, 41, 89, 23, 75
    img = torch.rand((B, Hs, Ws, C), generator=g)
    Ks = configs.f32([configs.intrinsics_matrix(55.0, 57.0, 44.0, 20.0)] * B)
    Kt = configs.f32([configs.intrinsics_matrix(50.0, 49.0, 37.0, 11.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(2.5 * k - 1.0), (0.15 * k - 0.08, 0.02, -0.01))
                         for k in range(B)])
    depths = configs.inv_depths(0.9, 50, D)
    ki, proj = _host.psv_matrices(Ks, Kt, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Ht, Wt)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Ht, Wt)
    assert_bits(out.cpu().numpy(), want, f"C={C} D={D} shrink={shrink}")


@pytest.mark.parametrize("band", [1, 0])
@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("D", [10, 64])
def test_plane_sweep_band_ring_vs_oracle(C, D, band, dev, kopts):
    """The band-walking kernel's LDS ring over tall targets (several bands of 8 four-row tiles,
    a partial last band and segment): a view whose source rows slide down with the target rows
    (ring refills of a few rows), one tilted about x (windows that move faster than the tiles,
    reloads), one rotated by 90 degrees in-plane (a band's footprint sweeps the source
    sideways: the union column range is too wide for a ring, steps staged one by one) and a
    strongly perspective one (window heights changing along the band): bit-exact to the oracle."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    import math
    kopts(sweep_band=band, sweep_direct=-1)
    g = torch.Generator().manual_seed(400 + C + D)
    B, Hs, Ws, Ht, Wt = 4, 150, 190, 141, 133
    img = torch.rand((B, Hs, Ws, C), generator=g)
    K = configs.f32([configs.intrinsics_matrix(120.0, 118.0, 95.0, 75.0)] * B)

    def rot_x(deg):
        a = math.radians(deg)
        return [[1.0, 0.0, 0.0], [0.0, math.cos(a), -math.sin(a)], [0.0, math.sin(a), math.cos(a)]]

    def rot_z(deg):
        a = math.radians(deg)
        return [[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]]
    poses = configs.f32([configs.pose_from(configs.rot_y(1.0), (0.08, 0.01, 0.0)),
                         configs.pose_from(rot_x(12.0), (0.0, 0.1, 0.05)),
                         configs.pose_from(rot_z(90.0), (0.02, -0.03, 0.0)),
                         configs.pose_from(rot_x(-25.0), (0.05, 0.3, 0.6))])
    depths = configs.inv_depths(1, 60, D)
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Ht, Wt)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Ht, Wt)
    assert_bits(out.cpu().numpy(), want, f"C={C} D={D} band={band}")


@pytest.mark.parametrize("C", [3, 4])
def test_plane_sweep_depth_lanes_off_image(C, dev):
    """Depth-per-lane kernel on landscape sources with footprints wholly off the image (zero
    tiles and border-collapsed boxes), D = 64: bit-exact to the oracle, zeros included."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    g = torch.Generator().manual_seed(177 + C)
    B, Hs, Ws, D = 3, 60, 160, 64
    img = torch.rand((B, Hs, Ws, C), generator=g) + 0.5
    K = configs.f32([configs.intrinsics_matrix(150.0, 150.0, 80.0, 30.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(0.5), (0.1, 0.01, 0.0)),
                         configs.pose_from(configs.rot_y(-20.0), (1.5, 0.2, 0.1)),
                         configs.pose_from(configs.rot_y(40.0), (-2.0, -0.5, 0.3))])
    depths = configs.inv_depths(1, 50, D)
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Hs, Ws)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Hs, Ws)
    assert_bits(out.cpu().numpy(), want, f"C={C}")
    assert (want == 0).mean() > 0.2


def test_format_network_input_depth_lanes_strided(small, dev, kopts):
    """format_network_input_torch with 64 planes: every source swept by the depth-per-lane
    kernel straight from its strided channel slice into its channel slice of the network
    input (mpiv_plane_sweep_into), bit-identical to per-source volumes of the pixel-per-lane
    kernel on padded copies (itself pinned by the reference golden of
    test_format_network_input) concatenated after the reference image."""
    from mpi_vision_amd import _host, _lib
    t = {k: torch.tensor(small[f"fni_{k}"]) for k in ("ref", "src", "ref_pose", "src_poses", "K")}
    planes = configs.inv_depths(1.0, 100.0, 64)
    got = mv.format_network_input_torch(None, t["ref"].to(dev), t["src"].to(dev), t["ref_pose"].to(dev),
                                        t["src_poses"].to(dev), planes, t["K"].to(dev)).cpu()
    kopts(sweep_dlane=0)
    S = t["src_poses"].shape[1]
    inv_ref = torch.inverse(t["ref_pose"])
    H, W = t["ref"].shape[1], t["ref"].shape[2]
    parts = [t["ref"]]
    for i in range(S):
        ki, proj = _host.psv_matrices(t["K"], t["K"], torch.matmul(t["src_poses"][:, i], inv_ref))
        src = t["src"][..., i * 3:(i + 1) * 3].contiguous().to(dev)
        parts.append(_lib.plane_sweep_padded(src, planes, ki, proj, H, W).cpu())
    assert_bits(got.numpy(), torch.cat(parts, dim=-1).numpy())


@pytest.mark.parametrize("direct", ["0", "1", "2", "3"])
@pytest.mark.parametrize("D", [3, 6, 8, 10, 16])
def test_format_network_input_few_depths_routes(D, direct, small, dev, kopts):
    """format_network_input_torch with the notebook's few depths: each source swept into its
    channel slice of the network input (mpiv_plane_sweep_into: pixel runs D*3 floats long,
    out_pstride = 3 + S*D*3 apart) by the automatic route (D = 3..8: the pixel-per-lane kernel,
    ADVICE r3), the direct depth-per-lane kernel and the pixel-per-lane kernel (strided
    copy-out): bit-identical to the LDS-staged kernel (sweep_direct=-1)."""
    t = {k: torch.tensor(small[f"fni_{k}"]).to(dev) for k in ("ref", "src", "ref_pose", "src_poses", "K")}
    planes = configs.inv_depths(1.0, 100.0, D)
    args = (None, t["ref"], t["src"], t["ref_pose"], t["src_poses"], planes, t["K"])
    kopts(sweep_direct="-1")
    want = mv.format_network_input_torch(*args).cpu()
    kopts(sweep_direct=direct)
    got = mv.format_network_input_torch(*args).cpu()
    assert_bits(got.numpy(), want.numpy(), f"D={D} direct={direct}")


@pytest.mark.parametrize("shape", [(1, 1, 1, 1), (2, 3, 1, 2), (5, 4, 3, 65)])
def test_plane_sweep_tiny_targets(shape, dev):
    """Tiny targets and depth counts through the default (depth-per-lane, in-place) sweep:
    1x1 target with one depth and one channel, 2x3 targets, 65 depths (a one-depth second
    chunk) into a 5x4 target: bit-exact to the oracle."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    Ht, Wt, C, D = shape
    g = torch.Generator().manual_seed(200 + D)
    B, Hs, Ws = 2, 9, 11
    img = torch.rand((B, Hs, Ws, C), generator=g)
    Ks = configs.f32([configs.intrinsics_matrix(9.0, 9.5, 5.0, 4.0)] * B)
    Kt = configs.f32([configs.intrinsics_matrix(3.0, 3.0, Wt / 2.0, Ht / 2.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(3.0 * k - 1.0), (0.1 * k, 0.02, 0.0)) for k in range(B)])
    depths = configs.inv_depths(1.0, 20, D) if D > 1 else [2.5]
    ki, proj = _host.psv_matrices(Ks, Kt, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Ht, Wt)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Ht, Wt)
    assert_bits(out.cpu().numpy(), want, str(shape))


@pytest.mark.parametrize("C", [1, 2, 3, 4])
@pytest.mark.parametrize("D,direct", [(1, "0"), (6, "0"), (8, "0"), (10, "0"), (10, "1"), (16, "1"), (32, "1"), (33, "1"),
                                      (64, "1"), (1, "2"), (5, "2"), (10, "2"), (12, "2"), (16, "2"), (1, "3"), (7, "3"), (10, "3"),
                                      (16, "3")])
@pytest.mark.parametrize("strided", [False, True])
def test_plane_sweep_direct_vs_oracle(C, D, direct, strided, dev, kopts):
    """Few depths skip the LDS staging: the direct depth-per-lane kernel (automatic for D <= 2,
    sweep_direct=1 forces it up to D = 64) and the pixel-per-lane kernel plane_sweep_px_kernel
    (automatic for 3 <= D <= 8; sweep_direct=2 / 3 force it with 64 / 32 pixels per wave for
    D * C <= 48, the LDS kernel above); -1 keeps the LDS kernel.  Partial pixel groups
    (64 % D idle lanes, a partial last group of a row), odd target sizes, separate source /
    target intrinsics, a strided (channel-sliced) source: bit-exact to the oracle."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    kopts(sweep_direct=direct)
    g = torch.Generator().manual_seed(300 + C + D)
    B, Hs, Ws, Ht, Wt = 2, 37, 83, 29, 71
    full = torch.rand((B, Hs, Ws, C + 2), generator=g)
    img = full[..., 1:C + 1] if strided else full[..., :C].contiguous()
    Ks = configs.f32([configs.intrinsics_matrix(52.0, 55.0, 41.0, 19.0)] * B)
    Kt = configs.f32([configs.intrinsics_matrix(48.0, 47.0, 35.0, 14.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(3.0 * k - 1.5), (0.2 * k - 0.1, -0.03, 0.02))
                         for k in range(B)])
    depths = configs.inv_depths(0.8, 60, D) if D > 1 else [3.0]
    ki, proj = _host.psv_matrices(Ks, Kt, poses)
    want = oracle.plane_sweep(img.contiguous().numpy(), ki.numpy(), proj.numpy(), depths, Ht, Wt)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Ht, Wt)
    assert_bits(out.cpu().numpy(), want, f"C={C} D={D} direct={direct} strided={strided}")
    if direct == "0":  # mpiv_route reports production routes only
        _lib.reset_debug()
        route = _lib.route("plane_sweep", B, Hs, Ws, C, D, Ht, Wt)[0]
        want_route = ("plane_sweep_direct_kernel" if D <= 2 else "plane_sweep_px_kernel" if D <= 8
                      else "plane_sweep_dlane_kernel")
        assert route.startswith(want_route), route


@pytest.mark.parametrize("direct", ["0", "-1", "2", "3"])
def test_plane_sweep_direct_off_image(direct, dev, kopts):
    """The notebook's 10 planes on landscape sources whose samples fall wholly or partly off
    the image (the swapped x / H normalisation), through the direct kernel and the LDS kernel:
    bit-exact to the oracle, zeros included."""
    from mpi_vision_amd import _host, _lib
    from oracle import oracle
    kopts(sweep_direct=direct)
    g = torch.Generator().manual_seed(321)
    B, Hs, Ws, D = 3, 60, 160, 10
    img = torch.rand((B, Hs, Ws, 3), generator=g) + 0.5
    K = configs.f32([configs.intrinsics_matrix(150.0, 150.0, 80.0, 30.0)] * B)
    poses = configs.f32([configs.pose_from(configs.rot_y(0.5), (0.1, 0.01, 0.0)),
                         configs.pose_from(configs.rot_y(-20.0), (1.5, 0.2, 0.1)),
                         configs.pose_from(configs.rot_y(40.0), (-2.0, -0.5, 0.3))])
    depths = configs.inv_depths(1, 100, D)
    ki, proj = _host.psv_matrices(K, K, poses)
    want = oracle.plane_sweep(img.numpy(), ki.numpy(), proj.numpy(), depths, Hs, Ws)
    out = _lib.plane_sweep(img.to(dev), depths, ki, proj, Hs, Ws)
    assert_bits(out.cpu().numpy(), want, f"direct={direct}")
    assert (want == 0).mean() > 0.2

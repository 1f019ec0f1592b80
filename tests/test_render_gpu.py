"""GPU parity of the fused warp + over-composite kernels against the reference
goldens (bit-exact) and the CPU oracle (tests/golden/, tools/gen_goldens.py).

Tolerance: the bar is bit-exact (0 ulp) for every single-GPU render path; the
plane-sharded (C,T) reassociation is checked at 1e-5 absolute (BASELINE.json
north_star), with ~3e-7 expected."""
import numpy as np
import pytest
import torch

from conftest import RENDER_CASES, assert_bits, load_test_mpi, render_case_inputs, sha256

pytestmark = pytest.mark.gpu

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _lib, configs  # noqa: E402
from oracle import oracle  # noqa: E402


def _t(small, key, dev):
    return torch.tensor(small[key]).to(dev)


@pytest.mark.parametrize("name", RENDER_CASES)
def test_render_matches_reference(name, small, meta, dev):
    mpi = render_case_inputs(meta["small"], name)
    out = mv.mpi_render_view_torch(mpi.to(dev) if mpi.stride(0) else mpi[:1].to(dev).expand(*mpi.shape),
                                   _t(small, f"{name}_pose", dev), _t(small, f"{name}_depths", dev),
                                   _t(small, f"{name}_K", dev))
    assert_bits(out.cpu().numpy(), small[f"{name}_out"])


# in-place ([B,H,W,P,4]) kernels behind mpiv_render, selected by libmpiv's debug options
NATIVE_KERNELS = {"chunk8": dict(render_chunk=8, chunk_strip=0), "chunk4": dict(render_chunk=4),
                  "chunk8strip": dict(render_chunk=8, chunk_strip=1), "chunk8strip8": dict(render_chunk=8, chunk_strip=2),
                  "chunk8r2": dict(render_chunk=8, chunk_rows=2), "chunk8r4": dict(render_chunk=8, chunk_rows=4),
                  "chunk4r4": dict(render_chunk=4, chunk_rows=4),
                  "chunk8f4": dict(render_chunk=8, chunk_flight=4), "chunk4f4": dict(render_chunk=4, chunk_flight=4),
                  "lds": dict(render_chunk=-1, render_native_lds=1),
                  "direct": dict(render_chunk=-1, render_native_lds=0)}


@pytest.mark.parametrize("name", RENDER_CASES)
@pytest.mark.parametrize("native", list(NATIVE_KERNELS))
def test_native_and_packed_kernels_agree_with_oracle(name, native, small, meta, dev, kopts):
    """Both texel layouts (the in-place one through its chunked, direct and LDS-staged
    kernels), driven with the reference's own H bits."""
    kopts(**NATIVE_KERNELS[native])
    mpi = render_case_inputs(meta["small"], name)
    B, H, W, P, _ = mpi.shape
    homs = torch.tensor(small[f"{name}_H"]).permute(1, 0, 2, 3).reshape(B, P, 9).contiguous()
    want = oracle.render(mpi.numpy(), homs.numpy())
    dmpi = mpi.contiguous().to(dev)
    nat = torch.empty((B, H, W, 3), device=dev)
    _lib._call("mpiv_render", dmpi, _lib._strides(dmpi), B, H, W, P, homs.to(dev),
               nat, _lib._stream(dev))
    assert_bits(nat.cpu().numpy(), want)
    for b in range(B):
        packed = _lib.pack_planes(dmpi[b])
        want_pk = torch.zeros(_lib.packed_shape(H, W, P))
        want_pk[:, 2:2 + H, 2:2 + W] = mpi[b].permute(2, 0, 1, 3)
        assert torch.equal(packed.cpu(), want_pk)  # interior = plane-major texels, border = 0
        pk = _lib.render_packed(packed, homs[b:b + 1])
        assert_bits(pk.cpu().numpy(), want[b:b + 1])


def test_render_strided_views(small, meta, dev):
    """Non-contiguous MPI (a channel-sliced / permuted view) is read in place."""
    mpi = render_case_inputs(meta["small"], "render_a")
    big = torch.zeros((2, 72, 128, 8, 6))
    big[..., 1:5] = mpi
    dbig = big.to(dev)
    view = dbig[..., 1:5]
    out = mv.mpi_render_view_torch(view, _t(small, "render_a_pose", dev), _t(small, "render_a_depths", dev),
                                   _t(small, "render_a_K", dev))
    assert_bits(out.cpu().numpy(), small["render_a_out"])


def test_render_c1_test_mpi(large, meta, dev):
    """Config 1: the repo's 10-plane test MPI, two novel poses, full 400x640."""
    mpi = load_test_mpi()
    assert sha256(mpi) == meta["large"]["c1"]["mpi_sha"]
    dmpi = mpi.to(dev).expand(2, *mpi.shape[1:])
    out = mv.mpi_render_view_torch(dmpi, _t(large, "c1_pose", dev), _t(large, "c1_depths", dev),
                                   _t(large, "c1_K", dev))
    got = out.cpu().numpy()
    assert_bits(got, large["c1_out"])
    assert sha256(got) == meta["large"]["c1"]["out_sha"]
    # also the native (non-broadcast) kernel on each pose
    for b in range(2):
        o1 = mv.mpi_render_view_torch(mpi.to(dev), _t(large, "c1_pose", dev)[b:b + 1],
                                      _t(large, "c1_depths", dev), _t(large, "c1_K", dev)[b:b + 1])
        assert_bits(o1.cpu().numpy(), large["c1_out"][b:b + 1])


def test_render_c2_broadcast_batch(large, meta, dev):
    """Config 2 shapes (576x1024x32, MPI broadcast over the view batch)."""
    c2 = configs.config2()
    mpi = configs.synthetic_mpi(1, c2["H"], c2["W"], c2["P"], c2["seed"])
    assert sha256(mpi) == meta["large"]["c2"]["mpi_sha"]
    poses = _t(large, "c2_pose", dev)
    dmpi = mpi.to(dev).expand(poses.shape[0], *mpi.shape[1:])
    out = mv.mpi_render_view_torch(dmpi, poses, _t(large, "c2_depths", dev), _t(large, "c2_K", dev))
    assert sha256(out) == meta["large"]["c2"]["out_sha"]


@pytest.mark.parametrize("pose_index", [0, 500])
def test_render_c4_headline_config(pose_index, large, meta, dev):
    """Config 4 (the bench workload): 1024x1024x128 MPI, poses 0 and 500 of the path."""
    c4 = configs.config4()
    mpi = configs.synthetic_mpi(1, c4["H"], c4["W"], c4["P"], c4["seed"])
    assert sha256(mpi) == meta["large"]["c4"]["mpi_sha"]
    j = meta["large"]["c4"]["sel"].index(pose_index)
    out = mv.mpi_render_view_torch(mpi.to(dev), _t(large, f"c4_{pose_index}_pose", dev), _t(large, "c4_depths", dev),
                                   _t(large, "c4_K", dev))
    got = out.cpu().numpy().reshape(-1)
    np.testing.assert_array_equal(got[large[f"c4_{pose_index}_idx"]], large[f"c4_{pose_index}_val"])
    assert sha256(out) == meta["large"]["c4"]["out_sha"][j]


def test_plane_range_partials_combine(small, meta, dev):
    """(C,T) partials over plane ranges + ordered combine == sequential render (1e-5)."""
    mpi = render_case_inputs(meta["small"], "render_a")[0:1]
    P = mpi.shape[3]
    homs = torch.tensor(small["render_a_H"]).permute(1, 0, 2, 3)[0:1].reshape(1, P, 9).contiguous()
    packed = _lib.pack_planes(mpi[0].to(dev))
    want = small["render_a_out"][0:1]
    for cuts in ([0, 8], [0, 3, 8], [0, 1, 2, 5, 8], list(range(9))):
        parts = torch.stack([_lib.render_packed_ct(packed, homs, back=(a == 0), p_begin=a, p_end=b)
                             for a, b in zip(cuts[:-1], cuts[1:])])
        got = _lib.combine_ct(parts).cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)
        if len(cuts) == 2:
            assert_bits(got, want)  # a single range is the sequential order


def test_render_deterministic(small, meta, dev):
    mpi = render_case_inputs(meta["small"], "render_big").to(dev)
    args = (_t(small, "render_big_pose", dev), _t(small, "render_big_depths", dev), _t(small, "render_big_K", dev))
    a = mv.mpi_render_view_torch(mpi, *args)
    b = mv.mpi_render_view_torch(mpi, *args)
    assert torch.equal(a, b)


def test_render_errors(dev):
    mpi = torch.zeros((1, 8, 8, 2, 4), device=dev)
    pose = torch.eye(4, device=dev)[None]
    K = torch.eye(3, device=dev)[None]
    with pytest.raises(AttributeError):  # planes must be a tensor, like the reference
        mv.mpi_render_view_torch(mpi, pose, [2.0, 1.0], K)
    with pytest.raises(RuntimeError):
        mv.mpi_render_view_torch(mpi.double(), pose, torch.tensor([2.0, 1.0], device=dev), K)
    with pytest.raises(RuntimeError):  # batch mismatch
        mv.mpi_render_view_torch(mpi, pose.expand(2, 4, 4), torch.tensor([2.0, 1.0], device=dev), K.expand(2, 3, 3))
    # empty inputs: the reference raises RuntimeError for an empty batch, image or plane
    # stack (its reshapes / grid_sampler's non-empty check; measured), and so does the drop-in
    planes = torch.tensor([2.0, 1.0], device=dev)
    for bad in (lambda: mv.mpi_render_view_torch(mpi[:0], pose[:0], planes, K[:0]),
                lambda: mv.mpi_render_view_torch(mpi[:, :0], pose, planes, K),
                lambda: mv.mpi_render_view_torch(mpi[..., :0, :], pose, planes[:0], K)):
        with pytest.raises(RuntimeError):
            bad()


@pytest.mark.parametrize("divisor", [1, 2, 3, 7, 36, 39, 47, 48, 63, 64, 71, 95, 96, 127, 159, 255, 399, 400,
                                     575, 576, 639, 640, 767, 768, 1023, 1024, 1079, 2159, 4095, 65535])
def test_div_const_exhaustive(divisor, dev):
    """The render's launch-constant division equals IEEE x / c for every fp32 x whose
    quotient can affect a sample position (all 2^32 bit patterns)."""
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    _lib._call("mpiv_selftest_div_const", divisor, bad, _lib._stream(dev))
    assert int(bad.item()) == 0


@pytest.mark.parametrize("name", RENDER_CASES)
def test_lds_and_direct_kernels_identical(name, small, meta, dev):
    """The LDS-staged render and the direct-gather render (default) agree bit for bit,
    including planes that fall back to direct gathers (large motion, 'render_big')."""
    mpi = render_case_inputs(meta["small"], name)
    B, H, W, P, _ = mpi.shape
    homs = torch.tensor(small[f"{name}_H"]).permute(1, 0, 2, 3).reshape(B, P, 9).contiguous()
    for b in range(B):
        packed = _lib.pack_planes(mpi[b].contiguous().to(dev))
        h = homs[b:b + 1].to(dev)
        a = torch.empty((1, H, W, 3), device=dev)
        d = torch.empty((1, H, W, 3), device=dev)
        _lib._call("mpiv_render_packed_lds", packed, H, W, P, h, 1, a, _lib._stream(dev))
        _lib._call("mpiv_render_packed", packed, H, W, P, h, 1, d, _lib._stream(dev))
        assert_bits(a.cpu().numpy(), d.cpu().numpy(), f"{name}[{b}] lds vs direct")
        assert_bits(a.cpu().numpy(), small[f"{name}_out"][b:b + 1], f"{name}[{b}] lds vs reference")


def test_lds_kernel_extreme_poses(dev):
    """Random large rotations / translations / planes behind the camera: the LDS
    kernel (with its per-plane direct fallback) equals the oracle bit for bit."""
    g = torch.Generator().manual_seed(99)
    H, W, P, V = 70, 150, 9, 6
    mpi = configs.synthetic_mpi(1, H, W, P, 3)
    poses = []
    for k in range(V):
        ang = (k - 3) * 12.0
        t = ((torch.rand(3, generator=g) - 0.5) * (0.5 + k)).tolist()
        poses.append(configs.pose_from(configs.rot_y(ang), t))
    poses = configs.f32(poses)
    K = configs.f32([configs.intrinsics_matrix(90.0, 95.0, 70.0, 33.0)] * V)
    depths = configs.f32(configs.inv_depths(0.3, 30, P))
    from mpi_vision_amd import _host
    homs = _host.render_homographies(poses, depths, K, V)
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    packed = _lib.pack_planes(mpi[0].to(dev))
    got = _lib.render_packed(packed, homs)
    assert_bits(got.cpu().numpy(), want)
    out = torch.empty_like(got)
    _lib._call("mpiv_render_packed_lds", packed, H, W, P, homs.to(dev), V, out, _lib._stream(dev))
    assert_bits(out.cpu().numpy(), want)


def _multiview_case(V, seed=7):
    """A camera-path stretch plus large rotations / translations (planes partly behind
    the camera) on an odd-sized MPI: V views, homographies, oracle frames."""
    from mpi_vision_amd import _host
    g = torch.Generator().manual_seed(seed)
    H, W, P = 70, 150, 9
    mpi = configs.synthetic_mpi(1, H, W, P, 4)
    n_path = max(V - 5, 1)
    poses = [configs.pose_from(configs.rot_y(0.3 * k), (0.01 * k, -0.005 * k, 0.002 * k)) for k in range(n_path)]
    for k in range(V - n_path):
        t = ((torch.rand(3, generator=g) - 0.5) * (0.5 + k)).tolist()
        poses.append(configs.pose_from(configs.rot_y((k - 2) * 15.0), t))
    poses = configs.f32(poses)
    K = configs.f32([configs.intrinsics_matrix(90.0, 95.0, 70.0, 33.0)] * V)
    depths = configs.f32(configs.inv_depths(0.3, 30, P))
    homs = _host.render_homographies(poses, depths, K, V)
    return mpi, homs


@pytest.mark.parametrize("shrink", ["0", "2"])
def test_multiview_kernel_bit_exact(shrink, dev, kopts):
    """render_mv_kernel (debug option render_mv=1, >= 4 views per launch): 11 views = a full
    group of 8 + a partial one, bit-exact to the oracle and to the direct-gather kernel (the
    default).  box_shrink=2 stages every box 2 texels narrower per side than the
    footprint, which forces the per-sample global fallback on most samples."""
    kopts(box_shrink=shrink, render_mv=1)
    mpi, homs = _multiview_case(11)
    V, P = homs.shape[0], homs.shape[1]
    H, W = mpi.shape[1], mpi.shape[2]
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    packed = _lib.pack_planes(mpi[0].to(dev))
    assert_bits(_lib.render_packed(packed, homs).cpu().numpy(), want, "multi-view")
    kopts(render_mv=0)
    assert_bits(_lib.render_packed(packed, homs).cpu().numpy(), want, "direct")


def _variant_env(kopts, mv):
    """mv "0" / "1": direct / multi-view LDS kernel; "pair" / "pair1": the pixel-pair
    tap-sharing kernel with two / one planes in flight (A/B); "ring<k>": the LDS-DMA ring
    kernel with tile geometry k (render_ring.hip); "tile<R>": R rows per work-item
    (render_rows_kernel), "tile8vs": with vertical tap sharing."""
    if mv.startswith("vsd"):  # vertical reuse, (R, rows in flight) = (8, 4) / (6, 3) / (9, 3) / (4, 4)
        # suffix "s": same-row tap reuse forced on (square frames too), "n": off (stretched frames too)
        same = {"s": 1, "n": -1, "o": 2}.get(mv[-1], 0)  # "o": with the out-of-range south loads (OOB)
        kopts(render_vshare=int(mv[3:].rstrip("sno")), render_same=same)
        return
    kopts(render_mv=1 if mv == "1" else 0, render_pair={"pair": 1, "pair1": 2}.get(mv, 0),
          render_ring=int(mv[4:]) if mv.startswith("ring") else -1,
          render_tile=int(mv[4:].replace("vs", "")) if mv.startswith("tile") else -1,
          render_vshare=1 if mv.endswith("vs") else 0)


RING = ["ring1", "ring2", "ring3", "ring4", "ring5", "ring6", "ring7", "ring8", "tile2", "tile4", "tile8", "tile8vs", "vsd3", "vsd4", "vsd5", "vsd11",
        "vsd3s", "vsd4s", "vsd5s", "vsd11s", "vsd4n", "vsd5n", "vsd4o",
        "tile16",
        "tile108", "tile116", "tile132"]


@pytest.mark.parametrize("variant", ["pair", "pair1"] + RING)
def test_sharing_kernels_odd_width_and_extreme_poses(variant, dev, kopts):
    """The tap-sharing kernels on an odd width (the last pair has no second pixel; a
    partial wave), a partial tile and strongly minifying / magnifying views (neighbours
    that do not share their taps): bit-exact vs the oracle."""
    _variant_env(kopts, variant)
    from mpi_vision_amd import _host
    H, W, P, V = 37, 203, 7, 3
    mpi = configs.synthetic_mpi(1, H, W, P, 12)
    K = configs.f32([configs.intrinsics_matrix(90.0, 85.0, W / 2.0, H / 2.0)] * V)
    poses = configs.f32([configs.pose_from(configs.rot_y(12.0), (0.3, -0.1, 0.6)),
                         configs.pose_from(configs.rot_y(-3.0), (0.02, 0.01, -0.7)),
                         configs.pose_from(configs.rot_y(0.5), (0.01, 0.0, 0.0))])
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V)
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    got = _lib.render_packed(_lib.pack_planes(mpi[0].to(dev)), homs)
    assert_bits(got.cpu().numpy(), want)


@pytest.mark.parametrize("mv", ["0", "1", "pair", "pair1"] + RING)
def test_multiview_camera_path_many_views(mv, dev, kopts):
    """A config-4-style sway path (40 consecutive poses of the 1000-pose path, 24 planes,
    viewer camera) rendered in one launch by the direct and the multi-view kernel:
    bit-exact."""
    _variant_env(kopts, mv)
    from mpi_vision_amd import _host
    H, W, P, V = 96, 160, 24, 40
    mpi = configs.synthetic_mpi(1, H, W, P, 9)
    f = configs.focal_from_fov(W)
    poses = configs.f32(configs.sway_path(1000)[100:100 + V])
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V)
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    got = _lib.render_packed(_lib.pack_planes(mpi[0].to(dev)), homs)
    assert_bits(got.cpu().numpy(), want)


@pytest.mark.parametrize("mv", ["0", "1", "pair", "pair1"] + RING)
def test_multiview_ct_partials(mv, dev, kopts):
    """Plane-range (C, T) partials of 6 views (direct and multi-view kernel) equal the
    oracle's bit for bit, and their ordered combine equals the sequential render (1e-5)."""
    _variant_env(kopts, mv)
    mpi, homs = _multiview_case(6, seed=3)
    V, P = homs.shape[0], homs.shape[1]
    H, W = mpi.shape[1], mpi.shape[2]
    full = mpi.expand(V, H, W, P, 4).numpy()
    packed = _lib.pack_planes(mpi[0].to(dev))
    cuts = [0, 4, 7, P]
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        ct = _lib.render_packed_ct(packed, homs, back=(a == 0), p_begin=a, p_end=b)
        assert_bits(ct.cpu().numpy(), oracle.render_ct(full, homs.numpy(), a, b, back=(a == 0)), f"ct [{a},{b})")
        parts.append(ct)
    got = _lib.combine_ct(torch.stack(parts)).cpu().numpy()
    np.testing.assert_allclose(got, oracle.render(full, homs.numpy()), rtol=0, atol=1e-5)


def _chunk_case(H, W, P, V, seed):
    """V views of V different MPIs (non-broadcast, the training caller's layout) from large
    rotations / translations (planes partly behind the camera, taps far off the image)."""
    from mpi_vision_amd import _host
    g = torch.Generator().manual_seed(seed)
    mpi = configs.synthetic_mpi(V, H, W, P, seed)
    poses = [configs.pose_from(configs.rot_y(0.2), (0.01, 0.0, 0.0))]
    for k in range(V - 1):
        t = ((torch.rand(3, generator=g) - 0.5) * (0.4 + k)).tolist()
        poses.append(configs.pose_from(configs.rot_y((k - 2) * 11.0), t))
    K = configs.f32([configs.intrinsics_matrix(90.0, 85.0, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(configs.f32(poses), configs.f32(configs.inv_depths(0.5, 50, P)), K, V)
    return mpi, homs


CHUNK_ROWS = {1: dict(chunk_strip=0), 2: dict(chunk_rows=2), 4: dict(chunk_rows=4), "f4": dict(chunk_flight=4),
              "strip": dict(chunk_strip=1), "strip8": dict(chunk_strip=2), "strip_n3": dict(chunk_strip=3),
              "strip16_n3": dict(chunk_strip=4)}


@pytest.mark.parametrize("rows", list(CHUNK_ROWS))
@pytest.mark.parametrize("ch", [4, 8])
@pytest.mark.parametrize("shape", [(37, 203, 13), (70, 150, 9), (33, 64, 8), (21, 70, 3), (5, 130, 21)])
def test_chunk_kernel_odd_shapes_extreme_poses(ch, rows, shape, dev, kopts):
    """render_chunk_kernel: plane counts that leave a partial last chunk, partial tiles in
    x and y (and a wave's row group past the frame), non-broadcast batches and extreme views,
    at 1, 2 and 4 rows per wave, with 4 sub-steps in flight ("f4") and as 8 x 16 / 8 x 8 strips with
    vertical tap reuse ("strip*", CH = 8 only): bit-exact vs the oracle."""
    kopts(render_chunk=ch, **CHUNK_ROWS[rows])
    H, W, P = shape
    mpi, homs = _chunk_case(H, W, P, 5, seed=H + W + P)
    want = oracle.render(mpi.numpy(), homs.numpy())
    dmpi = mpi.to(dev)
    out = torch.empty((5, H, W, 3), device=dev)
    _lib._call("mpiv_render", dmpi, _lib._strides(dmpi), 5, H, W, P, homs.to(dev), out, _lib._stream(dev))
    assert_bits(out.cpu().numpy(), want)


def test_chunk_kernel_plane_and_pixel_strides(dev):
    """The drop-in on a plane-sliced / cropped view of a larger tensor (planes still
    contiguous per pixel, pixel and row strides larger than P*4): the chunked kernel reads
    it in place, bit-exact vs the oracle on the same values."""
    H, W, P = 40, 72, 11
    big = configs.synthetic_mpi(2, H + 3, W + 5, P + 6, 21)
    view = big.to(dev)[:, 1:1 + H, 2:2 + W, 3:3 + P, :]
    assert _lib.chunk_layout_ok(view) and not view.is_contiguous()
    _, homs = _chunk_case(H, W, P, 2, seed=5)
    want = oracle.render(big[:, 1:1 + H, 2:2 + W, 3:3 + P, :].contiguous().numpy(), homs.numpy())
    out = torch.empty((2, H, W, 3), device=dev)
    _lib._call("mpiv_render", view, _lib._strides(view), 2, H, W, P, homs.to(dev), out, _lib._stream(dev))
    assert_bits(out.cpu().numpy(), want)


@pytest.mark.parametrize("ring", RING)
@pytest.mark.parametrize("name", RENDER_CASES)
def test_ring_kernel_golden_cases(ring, name, small, meta, dev, kopts):
    """The LDS-DMA ring render on the reference golden cases (incl. 'render_big': planes
    whose footprints do not fit a slot render direct) and on extreme views: bit-exact."""
    _variant_env(kopts, ring)
    mpi = render_case_inputs(meta["small"], name)
    B, H, W, P, _ = mpi.shape
    homs = torch.tensor(small[f"{name}_H"]).permute(1, 0, 2, 3).reshape(B, P, 9).contiguous()
    for b in range(B):
        packed = _lib.pack_planes(mpi[b].contiguous().to(dev))
        got = _lib.render_packed(packed, homs[b:b + 1])
        assert_bits(got.cpu().numpy(), small[f"{name}_out"][b:b + 1], f"{name}[{b}]")
    mpi, homs = _multiview_case(6, seed=11)
    V, P = homs.shape[0], homs.shape[1]
    H, W = mpi.shape[1], mpi.shape[2]
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    assert_bits(_lib.render_packed(_lib.pack_planes(mpi[0].to(dev)), homs).cpu().numpy(), want, "extreme views")


@pytest.mark.parametrize("V", [1, 2, 3, 9, 40])
def test_default_routing_square_camera_path(V, dev):
    """Default routing on a square MPI (render_rows_kernel with vertical tap reuse, (R, rows in
    flight) = (4, 4) at 1-2 views, (8, 4) up to 8, (6, 3) above) along the sway path, a frame
    height that is not a multiple of the block tile: bit-exact to the oracle."""
    from mpi_vision_amd import _host
    H, W, P = 100, 100, 16
    mpi = configs.synthetic_mpi(1, H, W, P, 21)
    f = configs.focal_from_fov(W)
    poses = configs.f32(configs.sway_path(1000)[300:300 + V])
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V)
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    got = _lib.render_packed(_lib.pack_planes(mpi[0].to(dev)), homs)
    assert_bits(got.cpu().numpy(), want)


@pytest.mark.parametrize("vs", ["-1", "1"])
def test_gather_census(vs, dev, kopts):
    """mpiv_render_packed_census (the counting build of render_rows_kernel, bench.py's texture
    roofline): same frames as the production launch; without vertical reuse exactly
    4 x (R*P + 1) gathers per wave, with it between 2 and 4 per plane-sample."""
    from mpi_vision_amd import _host
    kopts(render_tile=8, render_vshare=vs)
    H, W, P, V = 128, 128, 12, 5  # square: no tile samples the border alone (tile_dead)
    mpi = configs.synthetic_mpi(1, H, W, P, 4)
    f = configs.focal_from_fov(W)
    poses = configs.f32(configs.sway_path(1000)[40:40 + V])
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V).to(dev)
    packed = _lib.pack_planes(mpi[0].to(dev))
    want = _lib.render_packed(packed, homs)
    out = torch.empty_like(want)
    census = torch.zeros(1, dtype=torch.int64, device=dev)
    _lib._call("mpiv_render_packed_census", packed, H, W, P, homs, V, out, census, _lib._stream(dev))
    torch.cuda.synchronize()
    assert_bits(out.cpu().numpy(), want.cpu().numpy())
    waves = V * (W // 64) * (H // 8)
    n = int(census.item())
    if vs == "-1":
        assert n == waves * 4 * (8 * P + 1)
    else:
        assert waves * (2 * 8 * P + 2) <= n < waves * 4 * (8 * P + 1)


@pytest.mark.parametrize("V,R,D", [(1, 4, 4), (5, 8, 4), (12, 6, 3)])
def test_gather_census_default_routing(V, R, D, dev):
    """The counting build of the default route (vertical reuse, R rows with D in flight; a frame
    height that leaves a partial last tile): the production frames, and between 2 and 4
    gathers per computed plane-sample."""
    from mpi_vision_amd import _host
    H, W, P = 128, 128, 12  # square: the stretched route of a launch this small is the one-row kernel
    mpi = configs.synthetic_mpi(1, H, W, P, 4)
    f = configs.focal_from_fov(W)
    poses = configs.f32(configs.sway_path(1000)[40:40 + V])
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V).to(dev)
    packed = _lib.pack_planes(mpi[0].to(dev))
    want = _lib.render_packed(packed, homs)
    out = torch.empty_like(want)
    census = torch.zeros(1, dtype=torch.int64, device=dev)
    _lib._call("mpiv_render_packed_census", packed, H, W, P, homs, V, out, census, _lib._stream(dev))
    torch.cuda.synchronize()
    assert_bits(out.cpu().numpy(), want.cpu().numpy())
    waves = V * (W // 64) * ((H + R - 1) // R)  # waves whose first row is inside the frame
    n = int(census.item())
    assert waves * 2 * R * P <= n <= waves * 4 * (R * P + D)


def test_default_routing_stretched_many_views(dev):
    """Default routing on a stretched MPI (x footprints stretched by W/(H-1)) with enough views
    for the rows kernel (>= 2048 tiles of 64x32): R = 9 with 3 rows in flight, a frame height
    that leaves a partial tile: bit-exact to the oracle."""
    from mpi_vision_amd import _host
    H, W, P, V = 70, 256, 4, 200
    mpi = configs.synthetic_mpi(1, H, W, P, 23)
    f = configs.focal_from_fov(W)
    poses = configs.f32(configs.sway_path(1000)[500:500 + V])
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V)
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.numpy())
    got = _lib.render_packed(_lib.pack_planes(mpi[0].to(dev)), homs)
    assert_bits(got.cpu().numpy(), want)


@pytest.mark.parametrize("V", [1, 8, 64])
def test_same_row_reuse_census_and_frames(V, dev, kopts):
    """Same-row tap reuse (render.hip SAME) on a config-2-shaped stretched frame (the sample advances
    ~0.55 texel rows per output row): the default route's frames equal the oracle's and the frames
    without it (render_same=-1) bit for bit, and its counting build issues fewer gathers."""
    from mpi_vision_amd import _host
    H, W, P = 72, 128, 6
    mpi = configs.synthetic_mpi(1, H, W, P, 31)
    f = configs.focal_from_fov(W)
    poses = configs.f32(configs.sway_path(1000)[200:200 + V])
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V).to(dev)
    packed = _lib.pack_planes(mpi[0].to(dev))
    want = oracle.render(mpi.expand(V, H, W, P, 4).numpy(), homs.cpu().numpy())
    counts = {}
    for same in (2, 1, 0, -1):  # with OOB, without, automatic (OOB at one view), off
        kopts(render_vshare=4, render_same=same)
        assert_bits(_lib.render_packed(packed, homs).cpu().numpy(), want, f"render_same={same}")
        out = torch.empty((V, H, W, 3), device=dev)
        census = torch.zeros(1, dtype=torch.int64, device=dev)
        _lib._call("mpiv_render_packed_census", packed, H, W, P, homs, V, out, census, _lib._stream(dev))
        torch.cuda.synchronize()
        assert_bits(out.cpu().numpy(), want, f"census build, render_same={same}")
        counts[same] = int(census.item())
    # columns past ~H sample the zero border alone (tile_dead): those waves gather nothing
    waves = V * (W // 64) * (H // 6)
    assert 0 < counts[1] < counts[-1] <= waves * 4 * (6 * P + 3)
    assert counts[2] == counts[1] and counts[0] == counts[2 if V <= 2 else 1]  # OOB loads count as issued


@pytest.mark.parametrize("route", ["one_row", "rows"])
def test_dead_tiles_bit_exact(route, dev, kopts):
    """Tiles whose every sample reads the zero border (render.hip tile_dead: on a landscape MPI the
    reference's swapped normalisation sends every column past ~H there) take the zero-sample
    composite without positions or gathers: frames, (C, T) partials with and without the back plane
    and row bands equal the oracle bit for bit (signed zeros included), and the counting build shows
    the skipped gathers."""
    from mpi_vision_amd import _host
    if route == "rows":
        kopts(render_vshare=4)
    H, W, P, V = 54, 230, 9, 4
    mpi = configs.synthetic_mpi(1, H, W, P, 41)
    f = configs.focal_from_fov(W)
    poses = [configs.pose_from(configs.rot_y(0.0), (0.0, 0.0, 0.0))]
    poses += list(configs.sway_path(1000)[600:600 + V - 2])
    poses.append(configs.pose_from(configs.rot_y(20.0), (0.4, -0.2, 0.3)))  # planes sweep across the edge
    poses = configs.f32(poses)
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 100, P)), K, V)
    full = mpi.expand(V, H, W, P, 4).numpy()
    packed = _lib.pack_planes(mpi[0].to(dev))
    assert_bits(_lib.render_packed(packed, homs).cpu().numpy(), oracle.render(full, homs.numpy()), "frames")
    for a, b, back in ((0, 4, True), (4, P, False), (0, P, False)):
        ct = _lib.render_packed_ct(packed, homs, back=back, p_begin=a, p_end=b)
        assert_bits(ct.cpu().numpy(), oracle.render_ct(full, homs.numpy(), a, b, back=back), f"ct [{a},{b}) back={back}")
    if route == "rows":
        hd = homs.to(dev)
        out = torch.empty((V, H, W, 3), device=dev)
        census = torch.zeros(1, dtype=torch.int64, device=dev)
        _lib._call("mpiv_render_packed_census", packed, H, W, P, hd, V, out, census, _lib._stream(dev))
        torch.cuda.synchronize()
        waves = V * ((W + 63) // 64) * ((H + 5) // 6)
        assert int(census.item()) < waves * 2 * 6 * P  # fewer than every wave's minimum: whole tiles skipped

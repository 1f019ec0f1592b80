"""GPU parity of the 8-bit RGBA MPI render (render_u8.hip): frames from packed u8 texels
must equal the float render of u8.float() / 255 (the reference's image convention,
utils.py:324-331) BIT FOR BIT -- checked against the reference's own config-1 goldens
(its uint8 test MPI, tests/golden/test_mpi) and against the CPU oracle on random uint8
MPIs under extreme views, for both row depths of the kernel and the (C, T) partials."""
import numpy as np
import pytest
import torch

from conftest import assert_bits, load_test_mpi, sha256

pytestmark = pytest.mark.gpu

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib, configs  # noqa: E402
from mpi_vision_amd import utils as mvu  # noqa: E402
from oracle import oracle  # noqa: E402


def _test_mpi_u8():
    f = load_test_mpi()  # [1,400,640,10,4] = u8 / 255
    u8 = torch.round(f * 255).to(torch.uint8)
    assert torch.equal(u8.float() / 255, f)  # the PNG bytes, recovered exactly
    return u8


def _u8_to_float(u8: np.ndarray) -> np.ndarray:
    return u8.astype(np.float32) / np.float32(255.0)  # correctly rounded fp32 division



def _rows_opts(kopts, rows):
    """rows: 2 / 8 rows per lane, or "4vs" / "8vs": that many with vertical tap reuse (A/B);
    "4vsf2" / "4vsf4": 4 rows with reuse and 2 / 4 rows in flight (u8_flight); 0: automatic."""
    if isinstance(rows, str):
        n, _, f = rows.partition("vs")
        kopts(render_tile=int(n), render_vshare=1, **({"u8_flight": int(f[1:])} if f else {}))
    else:
        kopts(render_tile=rows)


@pytest.mark.parametrize("rows", [0, 2, 8, "4vs", "8vs", "4vsf2", "4vsf4", "4vsf8"])
def test_u8_render_reference_test_mpi(rows, large, meta, dev, kopts):
    """Config 1: the reference's 10-plane uint8 test MPI, two poses, against the goldens
    the reference produced from u8 / 255 (tools/gen_goldens.py)."""
    if rows:
        _rows_opts(kopts, rows)
    u8 = _test_mpi_u8().to(dev)
    pose = torch.tensor(large["c1_pose"]).to(dev)
    K = torch.tensor(large["c1_K"]).to(dev)
    depths = torch.tensor(large["c1_depths"]).to(dev)
    out = mvu.mpi_render_view_u8(u8.expand(2, *u8.shape[1:]), pose, depths, K)
    assert_bits(out.cpu().numpy(), large["c1_out"])
    assert sha256(out.cpu().numpy()) == meta["large"]["c1"]["out_sha"]
    for b in range(2):  # non-broadcast batch path (pack per view)
        o1 = mvu.mpi_render_view_u8(u8, pose[b:b + 1], depths, K[b:b + 1])
        assert_bits(o1.cpu().numpy(), large["c1_out"][b:b + 1])


def _extreme_case(V, H, W, P, seed):
    g = torch.Generator().manual_seed(seed)
    u8 = torch.randint(0, 256, (1, H, W, P, 4), generator=g, dtype=torch.uint8)
    u8[..., 0, 3] = 255
    poses = [configs.pose_from(configs.rot_y(0.3 * k), (0.01 * k, -0.005 * k, 0.002 * k)) for k in range(V - 3)]
    for k in range(3):
        t = ((torch.rand(3, generator=g) - 0.5) * (0.5 + k)).tolist()
        poses.append(configs.pose_from(configs.rot_y((k - 1) * 17.0), t))
    K = configs.f32([configs.intrinsics_matrix(90.0, 95.0, W / 2.0, H / 2.0)] * V)
    homs = _host.render_homographies(configs.f32(poses), configs.f32(configs.inv_depths(0.3, 30, P)), K, V)
    return u8, homs


@pytest.mark.parametrize("rows", [2, 8, "4vs", "8vs", "4vsf2", "4vsf4", "4vsf8"])
@pytest.mark.parametrize("shape", [(70, 150, 9), (37, 203, 7), (64, 66, 16)])
def test_u8_render_random_vs_oracle(rows, shape, dev, kopts):
    """Random bytes (every value 0..255 occurs), odd sizes, partial tiles, planes partly
    behind the camera: bit-exact vs the oracle on u8 / 255."""
    _rows_opts(kopts, rows)
    H, W, P = shape
    V = 7
    u8, homs = _extreme_case(V, H, W, P, seed=H * W + P)
    want = oracle.render(np.broadcast_to(_u8_to_float(u8.numpy()), (V, H, W, P, 4)).copy(), homs.numpy())
    packed = _lib.pack_planes_u8(u8[0].to(dev))
    assert_bits(_lib.render_packed_u8(packed, homs).cpu().numpy(), want)
    # the float path on the same values agrees too
    fl = torch.from_numpy(_u8_to_float(u8.numpy()))
    assert_bits(_lib.render_packed(_lib.pack_planes(fl[0].to(dev)), homs).cpu().numpy(), want, "float path")


@pytest.mark.parametrize("rows", [2, 8, "4vs", "8vs", "4vsf2", "4vsf4", "4vsf8"])
def test_u8_ct_partials(rows, dev, kopts):
    """Plane-range (C, T) partials of a u8 MPI equal the oracle's; their ordered combine
    equals the sequential render within 1e-5 (north_star)."""
    _rows_opts(kopts, rows)
    H, W, P, V = 45, 130, 11, 4
    u8, homs = _extreme_case(V, H, W, P, seed=5)
    full = np.broadcast_to(_u8_to_float(u8.numpy()), (V, H, W, P, 4)).copy()
    packed = _lib.pack_planes_u8(u8[0].to(dev))
    parts = []
    for a, b in zip([0, 3, 8], [3, 8, P]):
        ct = _lib.render_packed_u8_ct(packed, homs, back=(a == 0), p_begin=a, p_end=b)
        assert_bits(ct.cpu().numpy(), oracle.render_ct(full, homs.numpy(), a, b, back=(a == 0)), f"ct [{a},{b})")
        parts.append(ct)
    got = _lib.combine_ct(torch.stack(parts)).cpu().numpy()
    np.testing.assert_allclose(got, oracle.render(full, homs.numpy()), rtol=0, atol=1e-5)


def test_u8_pack_layout_and_strides(dev):
    """pack_planes_u8 = plane-major RGBA words with a zero border, for a strided view."""
    g = torch.Generator().manual_seed(2)
    big = torch.randint(0, 256, (9, 21, 6, 5), generator=g, dtype=torch.uint8)
    view = big.to(dev)[1:8, 2:19, 1:5, :4]  # [7, 17, 4, 4], channel stride 1, odd strides
    packed = _lib.pack_planes_u8(view)
    v = big[1:8, 2:19, 1:5, :4].to(torch.int64)
    words = (v[..., 0] | (v[..., 1] << 8) | (v[..., 2] << 16) | (v[..., 3] << 24)).permute(2, 0, 1)
    want = torch.zeros((4, 11, 21), dtype=torch.int64)
    want[:, 2:9, 2:19] = words
    got = packed.cpu().to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(got, want)


def test_u8_synth_shards_equal_whole(dev):
    """The counter-based u8 generator: plane ranges generated separately equal the same
    planes of the whole MPI (config-5 shards); plane 0 alpha = 255; zero border."""
    H, W, P = 33, 71, 9
    whole = _lib.synth_mpi_packed_u8(7, H, W, 0, P, dev)
    parts = torch.cat([_lib.synth_mpi_packed_u8(7, H, W, a, b, dev) for a, b in ((0, 2), (2, 5), (5, 9))])
    assert torch.equal(whole, parts)
    w = whole.cpu().to(torch.int64) & 0xFFFFFFFF
    assert torch.all((w[0, 2:2 + H, 2:2 + W] >> 24) == 255)
    assert torch.all(w[:, :2] == 0) and torch.all(w[:, :, -2:] == 0)
    assert len(torch.unique(w[1:, 2:2 + H, 2:2 + W] & 255)) == 256


def test_u8_render_rejects_unknown_row_variants(dev, kopts):
    """render_tile values the u8 render has no kernel for (4 rows without vertical reuse, 16)
    are refused instead of being silently remapped to another variant."""
    P, H, W = 3, 16, 70
    packed = _lib.synth_mpi_packed_u8(1, H, W, 0, P, dev)
    homs = torch.zeros((1, P, 9), device=dev)
    for rows in (4, 16):
        kopts(render_tile=rows)
        with pytest.raises(RuntimeError, match="not a u8 render variant"):
            _lib.render_packed_u8(packed, homs)


def test_u8_unpack_is_exact_float_of_every_byte(dev):
    """mpiv_unpack_planes_u8: every channel becomes RN(u8/255) (all 256 values, border zeros)."""
    H, W, P = 6, 16, 5
    g = torch.Generator().manual_seed(3)
    u8 = torch.randint(0, 256, (H, W, P, 4), generator=g, dtype=torch.uint8)
    u8.view(-1)[:256] = torch.arange(256, dtype=torch.int32).to(torch.uint8)
    pk = _lib.pack_planes_u8(u8.to(dev))
    f = _lib.unpack_planes_u8(pk)
    want = _lib.pack_planes((u8.float() / 255).to(dev))  # the float MPI's packed layout, same border
    assert_bits(f.cpu().numpy(), want.cpu().numpy(), "unpack")


def test_u8_many_views_route_through_float_copy(large, dev):
    """Launches of >= U8_FLOAT_MIN_VIEWS views render the MPI's exact float copy with the float
    kernel: the reference's config-1 goldens at 40 views (the two golden poses, 20 times each),
    and the same frames as the u8 kernel; the copy is made once per MPI (memo) and again after an
    in-place edit."""
    u8 = _test_mpi_u8().to(dev)
    V = 40
    assert V >= _lib.U8_FLOAT_MIN_VIEWS
    pose = torch.tensor(large["c1_pose"]).to(dev)[torch.arange(V) % 2]
    K = torch.tensor(large["c1_K"]).to(dev)[torch.arange(V) % 2]
    depths = torch.tensor(large["c1_depths"]).to(dev)
    out = mvu.mpi_render_view_u8(u8.expand(V, *u8.shape[1:]), pose, depths, K)
    assert_bits(out.cpu().numpy(), large["c1_out"][np.arange(V) % 2], "40 views of the golden poses")
    homs = _host.render_homographies(pose.cpu(), depths.cpu(), K.cpu(), V)
    pk = _lib.pack_planes_u8(u8[0])
    a = _lib.render_packed_u8(pk, homs, route_float=True)
    f1 = _lib.u8_float_copy(pk)
    assert _lib.u8_float_copy(pk) is f1  # memoised
    b = _lib.render_packed_u8(pk, homs, route_float=False)
    assert_bits(a.cpu().numpy(), b.cpu().numpy(), "float route vs u8 kernel")
    pk.view(torch.uint8)[..., 0] ^= 1  # in place: a new copy, new frames
    assert _lib.u8_float_copy(pk) is not f1
    c = _lib.render_packed_u8(pk, homs, route_float=True)
    d = _lib.render_packed_u8(pk, homs, route_float=False)
    assert_bits(c.cpu().numpy(), d.cpu().numpy(), "after an in-place edit")
    assert not torch.equal(a, c)


@pytest.mark.gpu
def test_u8_float_copy_follows_out_refills_streams_and_frees(dev, large):
    """refilling the same packed buffer through pack_planes_u8(out=) (a ctypes write,
    invisible to torch) must not render the old MPI's memoised float copy; a copy is not served to
    another stream; the memo entry goes when its u8 MPI is freed."""
    u8 = _test_mpi_u8().to(dev)
    V = 40
    pose = torch.tensor(large["c1_pose"]).to(dev)[torch.arange(V) % 2]
    K = torch.tensor(large["c1_K"]).to(dev)[torch.arange(V) % 2]
    depths = torch.tensor(large["c1_depths"]).to(dev)
    homs = _host.render_homographies(pose.cpu(), depths.cpu(), K.cpu(), V)
    pk = _lib.pack_planes_u8(u8[0])
    a = _lib.render_packed_u8(pk, homs, route_float=True)
    f1 = _lib.u8_float_copy(pk)
    other = u8[0].flip(0).contiguous()  # a different MPI of the same shape
    _lib.pack_planes_u8(other, out=pk)
    b = _lib.render_packed_u8(pk, homs, route_float=True)
    assert _lib.u8_float_copy(pk) is not f1
    assert not torch.equal(a, b)
    assert_bits(b.cpu().numpy(), _lib.render_packed_u8(pk, homs, route_float=False).cpu().numpy(),
                "refilled buffer: float route vs u8 kernel")
    f2 = _lib.u8_float_copy(pk)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        f3 = _lib.u8_float_copy(pk)
    s.synchronize()
    assert f3 is not f2 and torch.equal(f3, f2)
    del f1, f2, f3, pk
    assert dev not in _lib._U8_FLOAT
    _lib.clear_u8_float_copies()


@pytest.mark.gpu
def test_clear_u8_float_copies(dev):
    """The public release of the memoised float copies: per device and all devices."""
    u8 = _test_mpi_u8().to(dev)
    pk = _lib.pack_planes_u8(u8[0])
    _lib.u8_float_copy(pk)
    assert dev in _lib._U8_FLOAT
    _lib.clear_u8_float_copies(dev)
    assert dev not in _lib._U8_FLOAT
    _lib.u8_float_copy(pk)
    _lib.clear_u8_float_copies()
    assert not _lib._U8_FLOAT

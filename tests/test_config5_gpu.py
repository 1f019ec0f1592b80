"""BASELINE config 5 (256-plane 4096x2160 MPI, plane-sharded) at
full size on one MI355X: the 36.2 GB MPI fits in one GPU's HBM, so the sequential
render and the 8-shard (C, T) decomposition can be compared directly.

* The MPI is the counter-based synthetic one (synth.hip), generated on the device per
  plane range; oracle/mpiv_oracle.c restates the generator and renders any row band of
  the same MPI procedurally (no 36 GB host copy), so row bands are checked BIT-EXACT
  against the oracle (the reference recipe, pinned by tests/test_oracle.py).
* The 8 shards are generated separately (planes [32k, 32k+32)), rendered as (C, T)
  partials -- bit-exact to the oracle's partials on row bands -- and combined in plane
  order with mpiv_combine_ct: within 1e-5 of the sequential render everywhere
  (north_star tolerance; the reassociation moves results by ~1e-7).
"""
import numpy as np
import pytest
import torch

from conftest import assert_bits

pytestmark = pytest.mark.gpu

from mpi_vision_amd import _host, _lib, configs  # noqa: E402
from oracle import oracle  # noqa: E402

ROW_BANDS = [(0, 3), (537, 541), (1078, 1082), (1619, 1622), (2156, 2160)]


def _c5():
    c = configs.config5()
    homs = _host.render_homographies(configs.f32(c["poses"]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1)
    return c, homs


def test_synth_generator_matches_oracle_and_shards(dev):
    """The device generator equals the oracle's restatement bit for bit (packed layout,
    zero border included), and a plane range generated alone equals the same planes of
    the whole MPI."""
    H, W, P, seed = 37, 61, 9, 1234
    full = _lib.synth_mpi_packed(seed, H, W, 0, P, dev)
    want = torch.zeros(_lib.packed_shape(H, W, P))
    want[:, 2:2 + H, 2:2 + W] = torch.from_numpy(oracle.synth_mpi(seed, H, W, 0, P)).permute(2, 0, 1, 3)
    assert_bits(full, want.numpy(), "synthetic MPI")
    part = _lib.synth_mpi_packed(seed, H, W, 3, 7, dev)
    assert_bits(part, full[3:7].cpu().numpy(), "plane range 3..7")


def test_config5_full_size_sequential_and_plane_sharded(dev):
    c, homs = _c5()
    H, W, P, seed = c["H"], c["W"], c["P"], c["seed"]
    G = 8
    # sequential: all 256 planes (36.3 GB packed) in one launch
    packed = _lib.synth_mpi_packed(seed, H, W, 0, P, dev)
    frame = _lib.render_packed(packed, homs)
    torch.cuda.synchronize()
    del packed
    torch.cuda.empty_cache()
    frame_h = frame[0].cpu().numpy()
    assert np.isfinite(frame_h).all()
    for y0, y1 in ROW_BANDS:
        assert_bits(frame_h[y0:y1], oracle.render_synth(seed, H, W, homs[0].numpy(), y0, y1),
                    f"sequential rows {y0}..{y1}")
    # plane-sharded: G shards generated separately, (C, T) partials, ordered combine
    parts = torch.empty((G, 1, H, W, 4), device=dev)
    for k in range(G):
        p0, p1 = k * P // G, (k + 1) * P // G
        shard = _lib.synth_mpi_packed(seed, H, W, p0, p1, dev)
        _lib.render_packed_ct(shard, homs[:, p0:p1].contiguous(), back=(k == 0), out=parts[k])
        torch.cuda.synchronize()
        del shard
        y0, y1 = ROW_BANDS[k % len(ROW_BANDS)]
        assert_bits(parts[k, 0, y0:y1].cpu().numpy(),
                    oracle.render_synth(seed, H, W, homs[0].numpy(), y0, y1, p0=p0, p1=p1, back=(k == 0), ct=True),
                    f"shard {k} (C, T) rows {y0}..{y1}")
    combined = _lib.combine_ct(parts)[0].cpu().numpy()
    err = np.abs(combined.astype(np.float64) - frame_h).max()
    print(f"config 5: 8-shard combine vs sequential max |diff| = {err:.3g}")
    np.testing.assert_allclose(combined, frame_h, rtol=0, atol=1e-5)


@pytest.mark.parametrize("V,bands", [(1, 8), (1, 3), (3, 5), (12, 8)])
def test_ct_row_bands_equal_whole_partial(V, bands, dev):
    """mpiv_render_packed_ct_rows (the pipelined plane shard renders its row bands one launch
    each): the bands stitched together are bit-identical to one mpiv_render_packed_ct of the
    whole partial -- for a stretched frame (config 5's aspect, 1/8 size) and the back-most
    range (plane 0 replaces) and a middle range, at 1, 3 and 12 views."""
    from mpi_vision_amd import parallel
    c = configs.config5()
    H, W, P = 270, 512, 32
    K = configs.intrinsics_matrix(c["K"][0][0] / 8, c["K"][1][1] / 8, W / 2, H / 2)
    path = configs.config4()["poses"]
    homs = _host.render_homographies(configs.f32(path[10:10 + V]), configs.f32(configs.inv_depths(1, 100, P)),
                                     configs.f32([K] * V), V).to(dev)
    packed = _lib.synth_mpi_packed(7, H, W, 0, P, dev)
    for p0, p1, back in ((0, 12, True), (12, 32, False)):
        whole = _lib.render_packed_ct(packed, homs, back, p0, p1)
        banded = torch.full_like(whole, float("nan"))
        for b, e in parallel.band_bounds(H, bands):
            _lib.render_packed_ct_rows(packed, homs, back, b, e, banded, p0, p1)
        assert torch.equal(whole.view(torch.int32), banded.view(torch.int32)), (p0, p1)

"""Degenerate frame sizes (H or W = 1, 2x2) against goldens from the reference's own
mpi_render_view_torch (tools/gen_goldens_degenerate.py).  H = 1 or W = 1 divides by
H-1 = 0 or W-1 = 0 in the reference (utils.py:188), so its frames hold NaN; the oracle
and the HIP path must put NaN in the same places and match every other value bit for
bit (a NaN's payload is not part of the contract)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host  # noqa: E402

CASES = ["h1w7p3", "h5w1p3", "h2w2p2", "h1w1p2"]


@pytest.fixture(scope="module")
def degen():
    return np.load(os.path.join(GOLD, "degenerate.npz"))


def _match(got, want, what):
    got = np.ascontiguousarray(got, np.float32)
    want = np.ascontiguousarray(want, np.float32)
    assert got.shape == want.shape, what
    nan_g, nan_w = np.isnan(got), np.isnan(want)
    assert np.array_equal(nan_g, nan_w), f"{what}: NaN positions differ"
    assert np.array_equal(got[~nan_g].view(np.uint32), want[~nan_w].view(np.uint32)), f"{what}: values differ"


@pytest.mark.parametrize("tag", CASES)
def test_oracle_degenerate_sizes(tag, degen):
    from oracle import oracle
    homs = _host.render_homographies(torch.from_numpy(degen[tag + "_pose"]), torch.from_numpy(degen[tag + "_planes"]),
                                     torch.from_numpy(degen[tag + "_K"]), 1).numpy()
    _match(oracle.render(degen[tag + "_mpi"], homs), degen[tag + "_out"], tag)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", CASES)
def test_render_degenerate_sizes(tag, degen, dev):
    out = mv.mpi_render_view_torch(torch.from_numpy(degen[tag + "_mpi"]).to(dev),
                                   torch.from_numpy(degen[tag + "_pose"]).to(dev),
                                   torch.from_numpy(degen[tag + "_planes"]).to(dev),
                                   torch.from_numpy(degen[tag + "_K"]).to(dev))
    _match(out.cpu().numpy(), degen[tag + "_out"], tag)

"""GPU parity of the render BACKWARD (d render / d rgba_layers, render_bwd.hip) against
the reference's CPU autograd (tests/golden/grad.npz, tools/gen_goldens_grad.py) and
the oracle's restatement of it (oracle_render_backward, itself pinned bit-exact to
those goldens by tests/test_oracle.py).

Bar: bit-exact (0 ulp) for d rgba_layers, per view.  Two comparisons go through
torch's own GPU ops after our kernel and are toleranced (1e-6 absolute): the sum
over views that autograd's expand backward performs for a broadcast MPI, and the
notebook's training loss (mpi_from_net_output's elementwise ops + MSE)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD, assert_bits

pytestmark = pytest.mark.gpu

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib, configs  # noqa: E402
from oracle import oracle  # noqa: E402


@pytest.fixture(scope="module")
def grad():
    return np.load(os.path.join(GOLD, "grad.npz"))


# "tile": the production path (tile gather, pair count checked); "fallback": the bucket
# pipeline for every view (bwd_fallback=1); "miss": windows 1.5 px too small
# (bwd_margin=-96), so the tile gather misses contributors and the count must send every
# such view to the fallback; "barrier": the fallback on round 3's grid-barrier schedule
# (bwd_fb_mode=1, A/B) -- all bit-exact.  (The measured-and-rejected gather variants,
# bwd_gather=1|2|3, need an A/B build with one texel row per wave, -DMPIV_GTR=1.)
BWD_MODES = {"tile": {}, "fallback": {"bwd_fallback": 1}, "miss": {"bwd_margin": -96},
             "barrier": {"bwd_fallback": 1, "bwd_fb_mode": 1}}


@pytest.fixture(params=list(BWD_MODES))
def bwd_mode(request, kopts):
    kopts(**BWD_MODES[request.param])
    return request.param


def _backward_flag(mpi, homs, dout, dev):
    """(gradient, fallback flag of the last view) through a caller-owned workspace."""
    B, H, W, P, _ = mpi.shape
    L = _lib.load()
    ws = torch.zeros(L.mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    got = _lib.render_backward(mpi, homs, dout, workspace=ws)
    off = _lib.bwd_flag_offset(H, W, P)
    words = ws[off:off + 20].view(torch.int32).tolist()
    # words[1], [2]: the fallback's ticket and completion counters; [3], [4]: this view's /
    # this call's aborted fallbacks (a wait that outlasted its poll limit)
    assert words[3] == 0 and words[4] == 0, "the fallback aborted"
    assert _lib.render_backward_status(ws, H, W, P) == 0
    return got, words[0]


def _inputs(grad, name, dev):
    t = {k: torch.tensor(grad[f"{name}_{k}"]).to(dev) for k in ("pose", "K", "depths", "dout")}
    return torch.tensor(grad[f"{name}_mpi"]), t


@pytest.mark.parametrize("name", ["ga", "gbig", "gbin"])
def test_backward_matches_reference_autograd(name, grad, dev, bwd_mode):
    mpi, t = _inputs(grad, name, dev)
    leaf = mpi.to(dev).requires_grad_(True)
    out = mv.mpi_render_view_torch(leaf, t["pose"], t["depths"], t["K"])
    assert_bits(out.detach(), grad[f"{name}_out"], f"{name} forward")
    out.backward(t["dout"])
    assert_bits(leaf.grad, grad[f"{name}_grad"], f"{name} d rgba_layers")


def test_backward_collapsing_homography_vs_oracle(dev, bwd_mode):
    """Homographies that send many target pixels to one source texel: plane 0
    maps the whole frame to one point (one bucket holding every pixel), plane 1 minifies
    ~16x (buckets of ~70 pixels), plane 2 is a mild warp.  The large buckets take the
    block merge sort; the gradient stays bit-exact to the oracle's ordered scatter."""
    g = torch.Generator().manual_seed(17)
    H, W, P = 48, 80, 3
    mpi = configs.synthetic_mpi(1, H, W, P, 21)
    s = (H - 1) / (W - 1)  # the reference's swapped x / (H-1): undo it so the x step is 16 texels
    homs = torch.tensor([[[0.0, 0.0, 12.3, 0.0, 0.0, 7.6, 0.0, 0.0, 1.0],
                          [16.0 * s, 0.0, 0.5, 0.0, 16.0 / s, 0.25, 0.0, 0.0, 1.0],
                          [1.01, 0.02, -0.7, -0.01, 0.99, 0.4, 1e-4, 0.0, 1.0]]], dtype=torch.float32)
    dout = torch.rand((1, H, W, 3), generator=g) * 2 - 1
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    got = _lib.render_backward(mpi.to(dev), homs, dout.to(dev))
    assert_bits(got, want, "collapsing homographies")
    assert np.abs(want[0, :, :, 0]).max() > 1.0  # plane 0's one texel gathered the whole frame


def test_backward_one_bucket_at_config4_size(dev):
    """a legitimately slow fallback must complete, not time out into a NaN gradient.
    At config 4's size (1024 x 1024) plane 0 collapses the whole frame onto one texel -- ONE
    bucket of 2^20 pixels, which the fallback's phase 6 merge-sorts with a single block (its
    slowest case) while every other block waits on its ticket -- and plane 1 minifies 16x.
    The production path (tile gather refused -> fallback, wall-clock wait limit): no abort,
    the gradient bit-exact to the oracle."""
    g = torch.Generator().manual_seed(23)
    H = W = 1024
    P = 2
    mpi = configs.synthetic_mpi(1, H, W, P, 31)
    s = (H - 1) / (W - 1)
    homs = torch.tensor([[[0.0, 0.0, 511.3, 0.0, 0.0, 400.6, 0.0, 0.0, 1.0],
                          [16.0 * s, 0.0, 0.5, 0.0, 16.0 / s, 0.25, 0.0, 0.0, 1.0]]], dtype=torch.float32)
    dout = torch.rand((1, H, W, 3), generator=g) * 2 - 1
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    got, flag = _backward_flag(mpi.to(dev), homs, dout.to(dev), dev)
    assert flag == 1  # the view went through the fallback
    assert_bits(got, want, "one 2^20-pixel bucket")
    assert np.abs(want[0, :, :, 0]).max() > 100.0  # plane 0's one texel gathered the whole frame


def test_backward_broadcast_mpi(grad, dev, bwd_mode):
    """Broadcast MPI (stride-0 batch): per-view gradients are bit-exact to the oracle;
    their sum (torch's expand backward on the GPU) matches the reference within 1e-6."""
    mpi, t = _inputs(grad, "gbc", dev)
    B = t["dout"].shape[0]
    leaf = mpi.to(dev).requires_grad_(True)
    out = mv.mpi_render_view_torch(leaf.expand(B, *mpi.shape[1:]), t["pose"], t["depths"], t["K"])
    out.backward(t["dout"])
    np.testing.assert_allclose(leaf.grad.cpu().numpy(), grad["gbc_grad"], rtol=0, atol=1e-6)
    homs = grad["gbc_H"].transpose(1, 0, 2, 3).reshape(B, -1, 9)
    src = np.broadcast_to(grad["gbc_mpi"], (B,) + mpi.shape[1:])
    want = oracle.render_backward(src, homs, grad["gbc_dout"])
    per_view = _lib.render_backward(mpi.to(dev).expand(B, *mpi.shape[1:]), torch.tensor(homs), t["dout"])
    assert_bits(per_view, want, "per-view grads")


def test_backward_extreme_poses_vs_oracle(dev, bwd_mode):
    """Large rotations / translations, planes behind the camera, strong magnification and
    minification (buckets with many / no pixels): bit-exact to the oracle."""
    g = torch.Generator().manual_seed(5)
    H, W, P, V = 45, 71, 7, 5
    mpi = configs.synthetic_mpi(V, H, W, P, 8)
    poses = []
    for k in range(V):
        t = ((torch.rand(3, generator=g) - 0.5) * (0.4 + 1.2 * k)).tolist()
        poses.append(configs.pose_from(configs.rot_y((k - 2) * 15.0), t))
    poses = configs.f32(poses)
    K = configs.f32([configs.intrinsics_matrix(60.0 + 30 * k, 64.0, 35.0, 22.0) for k in range(V)])
    depths = configs.f32(configs.inv_depths(0.4, 20, P))
    homs = _host.render_homographies(poses, depths, K, V)
    dout = torch.rand((V, H, W, 3), generator=g) * 2 - 1
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    got = _lib.render_backward(mpi.to(dev), homs, dout.to(dev))
    assert_bits(got, want, "extreme poses")


def test_backward_medium_case_vs_oracle(dev, bwd_mode):
    """A 192x320x24 MPI over a camera-path pose: bit-exact to the oracle; the tile gather
    handles it without the fallback, and a too-small window is caught by the count."""
    H, W, P = 192, 320, 24
    mpi = configs.synthetic_mpi(1, H, W, P, 9)
    c = configs.config4()
    K = configs.f32([configs.intrinsics_matrix(277.0, 277.0, 160.0, 96.0)])
    homs = _host.render_homographies(configs.f32([c["poses"][123]]), configs.f32(configs.inv_depths(1, 100, P)),
                                     K, 1)
    dout = torch.rand((1, H, W, 3), generator=torch.Generator().manual_seed(3)) * 2 - 1
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    got, flag = _backward_flag(mpi.to(dev), homs, dout.to(dev), dev)
    assert_bits(got, want, "medium case")
    assert flag == (0 if bwd_mode == "tile" else 1)


def test_backward_deterministic(grad, dev):
    mpi, t = _inputs(grad, "ga", dev)
    homs = torch.tensor(grad["ga_H"]).permute(1, 0, 2, 3).reshape(2, 6, 9)
    a = _lib.render_backward(mpi.to(dev), homs, t["dout"])
    b = _lib.render_backward(mpi.to(dev), homs, t["dout"])
    assert torch.equal(a, b)


def _mpi_from_net_output(mpi_pred, ref_img, num_mpi_planes):
    """The notebook's MPI assembly (ipynb cell 10 L79-111) as broadcast torch ops on the
    GPU (same elementwise ops, so the same forward bits; autograd sums the background's
    gradient over planes in its own order, hence the 1e-6 tolerance below)."""
    p = mpi_pred.permute(0, 2, 3, 1)
    P = num_mpi_planes
    w = ((p[..., :P] + 1.) / 2.).unsqueeze(-1)
    alpha = ((p[..., P:2 * P] + 1.) / 2.).unsqueeze(-1)
    rgb = w * ref_img.unsqueeze(3) + (1 - w) * p[..., -3:].unsqueeze(3)
    return torch.cat([rgb, alpha], dim=-1)


def test_training_loss_gradient(grad, dev):
    """The notebook's test_loss (ipynb cell 12 L5-15) trained through the HIP renderer:
    the loss matches bit for bit, d loss / d network output within 1e-6."""
    pred = torch.tensor(grad["loss_pred"]).to(dev).requires_grad_(True)
    ref_img = torch.tensor(grad["loss_ref"]).to(dev)
    P = grad["loss_planes"].shape[0]
    rgba = _mpi_from_net_output(pred, ref_img, P)
    img = mv.mpi_render_view_torch(rgba, torch.tensor(grad["loss_pose"]).to(dev),
                                   torch.tensor(grad["loss_planes"]).to(dev), torch.tensor(grad["loss_K"]).to(dev))
    loss = torch.nn.functional.mse_loss(img, torch.tensor(grad["loss_tgt"]).to(dev))
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(grad["loss_value"]), rtol=1e-6)
    np.testing.assert_allclose(pred.grad.cpu().numpy(), grad["loss_grad"], rtol=0, atol=1e-6)


def test_training_loss_gradient_hip_assembly(grad, dev):
    """The same training loss with the MPI assembled by the HIP drop-in
    (mv.mpi_from_net_output, assemble.hip) instead of torch ops: loss and gradient
    through assembly + render + MSE against the reference's CPU autograd."""
    pred = torch.tensor(grad["loss_pred"]).to(dev).requires_grad_(True)
    P = grad["loss_planes"].shape[0]
    dep = {"mpi_planes": torch.zeros((pred.shape[0], P), device=dev),
           "ref_img": torch.tensor(grad["loss_ref"]).to(dev)}
    rgba = mv.mpi_from_net_output(pred, dep)
    img = mv.mpi_render_view_torch(rgba, torch.tensor(grad["loss_pose"]).to(dev),
                                   torch.tensor(grad["loss_planes"]).to(dev), torch.tensor(grad["loss_K"]).to(dev))
    loss = torch.nn.functional.mse_loss(img, torch.tensor(grad["loss_tgt"]).to(dev))
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(grad["loss_value"]), rtol=1e-6)
    np.testing.assert_allclose(pred.grad.cpu().numpy(), grad["loss_grad"], rtol=0, atol=1e-6)


def test_backward_strided_layout_vs_oracle(dev):
    """An MPI whose planes are not contiguous per pixel (a permuted [B,P,H,W,4] tensor) is
    made contiguous first; odd sizes (W % 8 != 0, partial plane chunk and gather group)."""
    H, W, P = 37, 53, 11
    base = configs.synthetic_mpi(1, H, W, P, 4)
    mpi = base.permute(0, 3, 1, 2, 4).contiguous().permute(0, 2, 3, 1, 4)
    assert mpi.stride(3) != 4
    c = configs.config4()
    K = configs.f32([configs.intrinsics_matrix(40.0, 40.0, 26.0, 18.0)])
    homs = _host.render_homographies(configs.f32([c["poses"][300]]), configs.f32(configs.inv_depths(1, 50, P)), K, 1)
    dout = torch.rand((1, H, W, 3), generator=torch.Generator().manual_seed(8)) * 2 - 1
    want = oracle.render_backward(base.numpy(), homs.numpy(), dout.numpy())
    got, flag = _backward_flag(mpi.to(dev), homs, dout.to(dev), dev)
    assert_bits(got, want, "strided layout")
    assert flag == 0


def test_backward_more_planes_than_lds_holds(dev):
    """P = 900 (> 796: the chain's homographies no longer fit beside its LDS slots, so it reads
    them from global memory; the training forward falls back to the plain render and the
    backward recomputes the composite): the drop-in's autograd equals the oracle bit for bit."""
    H, W, P = 12, 40, 900
    mpi = configs.synthetic_mpi(1, H, W, P, 6)
    c = configs.config4()
    K = configs.intrinsics_matrix(30.0, 30.0, 20.0, 6.0)
    planes = configs.f32(configs.inv_depths(1, 60, P))
    pose = configs.f32([c["poses"][120]])
    homs = _host.render_homographies(pose, planes, configs.f32([K]), 1)
    dout = torch.rand((1, H, W, 3), generator=torch.Generator().manual_seed(9)) * 2 - 1
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    leaf = mpi.to(dev).requires_grad_(True)
    out = mv.mpi_render_view_torch(leaf, pose.to(dev), planes.to(dev), configs.f32([K]).to(dev))
    out.backward(dout.to(dev))
    assert_bits(leaf.grad.cpu().numpy(), want, "P = 900")


@pytest.mark.parametrize("cfg", ["config2", "config4"])
def test_backward_full_size_tile_equals_fallback(cfg, dev, kopts):
    """BASELINE config 2 (1024x576x32, the stretched normalisation) and config 4
    (1024x1024x128) at full size: the tile gather takes every plane (flag 0) and its
    gradient is bit-identical to the bucket fallback's (the algorithm the small cases pin
    to the reference and the oracle)."""
    c = getattr(configs, cfg)()
    H, W, P = c["H"], c["W"], c["P"]
    g = torch.Generator(device=dev).manual_seed(11)
    mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c["poses"][7:8]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    fast, flag = _backward_flag(mpi, homs, dout, dev)
    assert flag == 0
    kopts(bwd_fallback=1)
    slow, flag = _backward_flag(mpi, homs, dout, dev)
    assert flag == 1
    assert torch.equal(fast.view(torch.int32), slow.view(torch.int32))


@pytest.mark.parametrize("rows", [1, 2, 4, "f4", "strip", "strip8", "strip_n3", "strip16_n3"])
@pytest.mark.parametrize("cfg", ["config2", "config4"])
def test_training_forward_checkpoints(cfg, rows, dev, kopts):
    """mpiv_render_train: frames bit-identical to the inference render; the backward fed its
    checkpoints (one pass) is bit-identical to the backward that recomputes them (two
    passes); two views in one launch (non-broadcast [2,H,W,P,4]); the forward at 1, 2 and 4
    rows per wave (chunk_rows), 4 sub-steps in flight and 8 x 16 / 8 x 8 strips with vertical tap reuse
    writes the same frames and checkpoints."""
    kopts(**{1: dict(chunk_strip=0), 2: dict(chunk_rows=2), 4: dict(chunk_rows=4), "f4": dict(chunk_flight=4),
             "strip": dict(chunk_strip=1), "strip8": dict(chunk_strip=2), "strip_n3": dict(chunk_strip=3),
             "strip16_n3": dict(chunk_strip=4)}[rows])
    c = getattr(configs, cfg)()
    H, W, P = c["H"], c["W"], c["P"]
    if cfg == "config4":
        H = W = 256  # full width of the pose set, fewer rows: two views stay small
    g = torch.Generator(device=dev).manual_seed(5)
    mpi = torch.rand((2, H, W, P, 4), generator=g, device=dev)
    K = configs.intrinsics_matrix(W * 0.9, W * 0.9, W / 2, H / 2)
    homs = _host.render_homographies(configs.f32(c["poses"][3:5]), configs.f32(c["depths"]), configs.f32([K, K]),
                                     2).to(dev)
    out, ck = _lib.render_train(mpi, homs)
    assert ck is not None and ck.shape == (2, (P + 7) // 8, H, W, 4)
    assert torch.equal(out.view(torch.int32), _lib.render(mpi, homs).view(torch.int32))
    dout = torch.rand((2, H, W, 3), generator=g, device=dev) * 2 - 1
    a = _lib.render_backward(mpi, homs, dout)
    b = _lib.render_backward(mpi, homs, dout, ckpt=ck)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def _medium_case(V=2):
    H, W, P = 64, 96, 12
    mpi = configs.synthetic_mpi(V, H, W, P, 19)
    c = configs.config4()
    K = configs.f32([configs.intrinsics_matrix(90.0, 90.0, 48.0, 32.0)] * V)
    homs = _host.render_homographies(configs.f32(c["poses"][40:40 + V]), configs.f32(configs.inv_depths(1, 80, P)),
                                     K, V)
    dout = torch.rand((V, H, W, 3), generator=torch.Generator().manual_seed(23)) * 2 - 1
    return mpi, homs, dout


def test_backward_fallback_more_blocks_than_resident(dev, kopts):
    """The fallback's phases are ordered by tickets, not by barriers over resident blocks
    (ADVICE r3): launched with 20000 blocks -- far more than the device holds at once, which a
    grid barrier could never release -- it completes, bit-exact to the oracle, nothing aborted.
    With one block (every item in turn) and a fixed item order (the barrier schedule expressed
    with the same counters) as well."""
    mpi, homs, dout = _medium_case()
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    for opts in ({"bwd_fb_blocks": 20000}, {"bwd_fb_blocks": 1}, {"bwd_fb_mode": 2, "bwd_fb_blocks": 8}):
        kopts(**{"bwd_fallback": 1, "bwd_fb_mode": 0, "bwd_fb_blocks": 0, **opts})
        got, flag = _backward_flag(mpi.to(dev), homs, dout.to(dev), dev)
        assert flag == 1
        assert_bits(got, want, f"fallback {opts}")


@pytest.mark.parametrize("blocks,nphase,nvirt", [(1, 9, 4), (4, 9, 4), (1024, 9, 1024), (20000, 9, 1024)])
def test_ticket_protocol_selftest(blocks, nphase, nvirt, dev):
    """The fallback's ticket schedule with trivial items (mpiv_selftest_tickets, libmpiv_ab.so):
    every item runs once, only after all items of the phase before it (no violation), nothing
    waits out its poll limit -- from one block to far more blocks than fit at once."""
    import ctypes
    L = _lib.load_ab()
    ctr = torch.zeros(4, dtype=torch.int32, device=dev)
    marks = torch.zeros(nphase * nvirt, dtype=torch.int32, device=dev)
    rc = L.mpiv_selftest_tickets(blocks, nphase, nvirt, 1 << 22, ctypes.c_void_p(ctr.data_ptr()),
                                 ctypes.c_void_p(marks.data_ptr()),
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, L.mpiv_last_error()
    c = ctr.tolist()
    assert c[1] == nphase * nvirt and c[2] == 0 and c[3] == 0, c
    assert int(marks.sum().item()) == nphase * nvirt


def test_backward_fallback_abort_is_loud(dev, kopts):
    """A fallback barrier wait that outlasts its poll limit (forced here at the first barrier,
    ADVICE r3: blocks kept from residency by other work on the device) never returns a
    plausible gradient: every aborted view is NaN, the status call counts them and
    render_backward(check=True) raises."""
    V = 2
    mpi, homs, dout = _medium_case(V)
    B, H, W, P, _ = mpi.shape
    kopts(bwd_fallback=1, bwd_poll_limit=-1)
    L = _lib.load()
    ws = torch.zeros(L.mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    got = _lib.render_backward(mpi.to(dev), homs, dout.to(dev), workspace=ws, check=False)
    assert _lib.render_backward_status(ws, H, W, P) == V
    assert torch.isnan(got).all()
    with pytest.raises(RuntimeError, match="aborted on 2 of 2 views"):
        _lib.render_backward(mpi.to(dev), homs, dout.to(dev), workspace=ws, check=True)
    # the production tile path on the same workspace: nothing aborted, the count starts over
    kopts(bwd_fallback=0, bwd_poll_limit=0)
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    got = _lib.render_backward(mpi.to(dev), homs, dout.to(dev), workspace=ws, check=True)
    assert_bits(got, want, "after an abort")


@pytest.mark.parametrize("ckpt", [True, False])
@pytest.mark.parametrize("mode", ["tile", "miss"])
def test_backward_launch_folded_schedule(ckpt, mode, dev, kopts):
    """Round 6: the one-group backward folds the counter memset and the planes' inverses into the
    box kernel (launched first), the pair-count check into the gather's last block and the
    aborted-view NaN fill into the fallback's last block (4 launches per view instead of 8).  Its
    gradient equals the unfolded schedule's (bwd_unfold=1) and the oracle bit for bit, over 3 views
    (counters reset between views), with and without checkpoints, with the tile gather complete and
    with induced misses (the folded check must send each view to the fallback); flag words agree."""
    V = 3
    mpi, homs, dout = _medium_case(V)
    B, H, W, P, _ = mpi.shape
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    m, h, d = mpi.to(dev), homs.to(dev), dout.to(dev)
    ck = _lib.render_train(m, h)[1] if ckpt else None
    if mode == "miss":
        kopts(bwd_margin=-96)
    L = _lib.load()
    res = {}
    for unfold in (0, 1):
        kopts(bwd_unfold=unfold)
        ws = torch.full((L.mpiv_render_backward_workspace_size(H, W, P),), 0x5A, dtype=torch.uint8, device=dev)
        got = _lib.render_backward(m, h, d, workspace=ws, ckpt=ck, check=True)
        off = _lib.bwd_flag_offset(H, W, P)
        res[unfold] = (got, ws[off:off + 40].view(torch.int32).tolist())
        assert_bits(got, want, f"unfold={unfold} {mode}")
    assert res[0][1][0] == res[1][1][0] == (1 if mode == "miss" else 0), (res[0][1], res[1][1])
    assert res[0][1][3:5] == res[1][1][3:5] == [0, 0]
    assert res[0][1][8:10] == [0, 0]  # the block-exit counters are left at zero for the next call


def test_backward_folded_abort_is_loud(dev, kopts):
    """The folded schedule's fallback (reached through induced misses, not forced) still poisons an
    aborted view from its last block: NaN gradient, counted, check=True raises (A/B: forced poll
    limit)."""
    V = 2
    mpi, homs, dout = _medium_case(V)
    B, H, W, P, _ = mpi.shape
    kopts(bwd_margin=-96, bwd_poll_limit=-1)
    L = _lib.load()
    ws = torch.zeros(L.mpiv_render_backward_workspace_size(H, W, P), dtype=torch.uint8, device=dev)
    got = _lib.render_backward(mpi.to(dev), homs, dout.to(dev), workspace=ws, check=False)
    assert _lib.render_backward_status(ws, H, W, P) == V
    assert torch.isnan(got).all()
    kopts(bwd_margin=16, bwd_poll_limit=0)
    got = _lib.render_backward(mpi.to(dev), homs, dout.to(dev), workspace=ws, check=True)
    assert_bits(got, oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy()), "after an abort")


def test_backward_abort_surfaces_on_next_default_call(dev, kopts):
    """the default render_backward (check=None, the autograd path) reads the abort
    count back asynchronously -- no synchronisation -- and the next call raises; so a training
    loop cannot keep stepping on NaN gradients.  render_backward_raise_pending waits and raises."""
    mpi, homs, dout = _medium_case(2)
    kopts(bwd_fallback=1, bwd_poll_limit=-1)
    leaf = mpi.to(dev).requires_grad_(True)
    out = _lib.RenderFunction.apply(leaf, homs.to(dev))
    out.backward(dout.to(dev))  # aborted (forced): NaN gradient, nothing raised yet
    assert torch.isnan(leaf.grad).all()
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="aborted on a view of an earlier backward"):
        _lib.render_backward(mpi.to(dev), homs, dout.to(dev))
    # the explicit wait-and-raise form
    _lib.render_backward(mpi.to(dev), homs, dout.to(dev))
    with pytest.raises(RuntimeError, match="earlier backward"):
        _lib.render_backward_raise_pending(dev)
    # production settings: no aborts, nothing raised, pending copies drain
    kopts(bwd_fallback=0, bwd_poll_limit=0)
    for _ in range(3):
        _lib.render_backward(mpi.to(dev), homs, dout.to(dev))
    _lib.render_backward_raise_pending(dev)


@pytest.mark.parametrize("group", [8, 16])
@pytest.mark.parametrize("overlap", [1, 0])
def test_backward_plane_groups_vs_oracle(group, overlap, dev, bwd_mode, kopts):
    """Plane groups (round 4: a view's backward runs group by group, back to front, the running
    adjoint handed down between groups, so the workspace holds one group's d samples): forced
    to 8 / 16 planes on a 36-plane MPI (5 / 3 groups, the last one partial), in every backward
    mode, with the forward's checkpoints (the drop-in's autograd) and without them (the
    checkpoints then come from a forward pass into the workspace): bit-exact vs the oracle."""
    H, W, P = 48, 80, 36
    mpi = configs.synthetic_mpi(1, H, W, P, 29)
    c = configs.config4()
    K = configs.intrinsics_matrix(70.0, 70.0, 40.0, 24.0)
    planes = configs.f32(configs.inv_depths(1, 70, P))
    pose = configs.f32([c["poses"][60]])
    homs = _host.render_homographies(pose, planes, configs.f32([K]), 1)
    dout = torch.rand((1, H, W, 3), generator=torch.Generator().manual_seed(31)) * 2 - 1
    want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
    # overlap 1 (round 5 default): group k's gather on a second stream beside group k-1's chain,
    # two d-sample windows; 0: the groups one after the other in one window
    kopts(bwd_group=group, bwd_overlap=overlap)
    L = _lib.load()
    assert L.mpiv_render_backward_workspace_size(H, W, P) < L.mpiv_render_backward_workspace_size(H, W, 2 * P)
    got, _ = _backward_flag(mpi.to(dev), homs, dout.to(dev), dev)  # no checkpoints
    assert_bits(got, want, f"groups of {group}, no checkpoints")
    leaf = mpi.to(dev).requires_grad_(True)
    out = mv.mpi_render_view_torch(leaf, pose.to(dev), planes.to(dev), configs.f32([K]).to(dev))
    out.backward(dout.to(dev))
    assert_bits(leaf.grad.cpu().numpy(), want, f"groups of {group}, forward checkpoints")
    # several views in one call: the schedule walks them in turn (the second stream's work of view v
    # is done before view v + 1 reuses the boxes and windows)
    mpi3 = configs.synthetic_mpi(3, H, W, P, 33)
    poses3 = configs.f32([c["poses"][60], c["poses"][300], c["poses"][700]])
    homs3 = _host.render_homographies(poses3, planes, configs.f32([K] * 3), 3)
    dout3 = torch.rand((3, H, W, 3), generator=torch.Generator().manual_seed(37)) * 2 - 1
    want3 = oracle.render_backward(mpi3.numpy(), homs3.numpy(), dout3.numpy())
    got3 = _lib.render_backward(mpi3.to(dev), homs3, dout3.to(dev), check=True)
    assert_bits(got3, want3, f"groups of {group}, 3 views")


def test_backward_config4_workspace_and_checkpoint_paths(dev):
    """Config 4 at full size in the smallest workspace (<= 1.5 GB, VERDICT r3: 4 plane groups of
    32 planes): the gradient equals the one-group run's (3.0 GB workspace) bit for bit, with the
    forward's checkpoints and with the checkpoints the backward computes itself (a forward pass
    into the workspace)."""
    c = configs.config4()
    H, W, P = c["H"], c["W"], c["P"]
    L = _lib.load()
    n_min = L.mpiv_render_backward_workspace_size_min(H, W, P)
    assert n_min <= 1.5e9 < L.mpiv_render_backward_workspace_size(H, W, P)
    g = torch.Generator(device=dev).manual_seed(13)
    mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
    homs = _host.render_homographies(configs.f32(c["poses"][200:201]), configs.f32(c["depths"]),
                                     configs.f32([c["K"]]), 1).to(dev)
    dout = torch.rand((1, H, W, 3), generator=g, device=dev) * 2 - 1
    _, ck = _lib.render_train(mpi, homs)
    one = _lib.render_backward(mpi, homs, dout, ckpt=ck, check=True)
    ws = torch.empty(n_min, dtype=torch.uint8, device=dev)
    a = _lib.render_backward(mpi, homs, dout, workspace=ws, ckpt=ck, check=True)
    del ck
    b = _lib.render_backward(mpi, homs, dout, workspace=ws, check=True)
    assert torch.equal(a.view(torch.int32), one.view(torch.int32))
    assert torch.equal(b.view(torch.int32), one.view(torch.int32))
    # the default workspace takes the overlapped schedule (4 groups, two windows, two streams); the
    # one-group sequential schedule gives the same bits
    with _lib.debug(bwd_overlap=0):
        seq = _lib.render_backward(mpi, homs, dout, check=True)
    assert torch.equal(seq.view(torch.int32), one.view(torch.int32))


class _RenderModule(torch.nn.Module):
    def __init__(self, pose, planes, K):
        super().__init__()
        self.pose, self.planes, self.K = pose, planes, K

    def forward(self, mpi):
        return mv.mpi_render_view_torch(mpi, self.pose, self.planes, self.K)


def test_training_step_captured_in_a_hip_graph(grad, dev):
    """The drop-in's training step (forward with checkpoints + the folded backward) captured in HIP graphs
    (torch.cuda.make_graphed_callables: every launch on the captured stream, no host synchronisation, the
    intrinsics inverse copied device to device inside the capture) and replayed: the reference's gradient
    bit for bit on every replay (golden 'ga')."""
    mpi, t = _inputs(grad, "ga", dev)
    leaf = mpi.to(dev).requires_grad_(True)
    graphed = torch.cuda.make_graphed_callables(_RenderModule(t["pose"], t["depths"], t["K"]), (leaf,))
    for _ in range(3):
        leaf.grad = None
        out = graphed(leaf)
        out.backward(t["dout"])
        torch.cuda.synchronize()
        assert_bits(leaf.grad, grad["ga_grad"], "graphed training step")
        assert_bits(out.detach(), grad["ga_out"], "graphed forward")


@pytest.mark.parametrize("group", [0, 8])
def test_backward_dead_tiles_vs_oracle(group, dev, bwd_mode, kopts):
    """Tiles whose samples all fall outside the image (render_bwd.hip bwd_chain_strip_kernel, round 6:
    on a landscape MPI the swapped normalisation sends every column past ~H there) skip the chain;
    with a pose whose planes sweep across the frame edge a tile can be dead for one plane group and
    live for another (the running adjoint handed down unchanged): bit-exact vs the oracle in every
    backward mode, one group and groups of 8 planes, with and without the forward's checkpoints."""
    H, W, P = 54, 230, 20
    mpi = configs.synthetic_mpi(1, H, W, P, 43)
    f = configs.focal_from_fov(W)
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)])
    planes = configs.f32(configs.inv_depths(0.5, 60, P))
    dout = torch.rand((1, H, W, 3), generator=torch.Generator().manual_seed(47)) * 2 - 1
    if group:
        kopts(bwd_group=group)
    for pose in (configs.pose_from(configs.rot_y(0.0), (0.0, 0.0, 0.0)),
                 configs.pose_from(configs.rot_y(14.0), (0.35, -0.1, 0.2))):
        pose = configs.f32([pose])
        homs = _host.render_homographies(pose, planes, K, 1)
        want = oracle.render_backward(mpi.numpy(), homs.numpy(), dout.numpy())
        got, _ = _backward_flag(mpi.to(dev), homs, dout.to(dev), dev)  # no checkpoints
        assert_bits(got, want, "no checkpoints")
        leaf = mpi.to(dev).requires_grad_(True)
        out = mv.mpi_render_view_torch(leaf, pose.to(dev), planes.to(dev), K.to(dev))
        out.backward(dout.to(dev))
        assert_bits(leaf.grad.cpu().numpy(), want, "forward checkpoints")

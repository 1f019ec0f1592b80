"""GPU parity of the MPI assembly from the network output (assemble.hip; the notebook's
mpi_from_net_output, ipynb cell 10 L79-111) against the notebook's own function run
on CPU with autograd (tests/golden/netout.npz, tools/gen_goldens_netout.py) and the
oracle's restatement (oracle.assemble_mpi[_backward], pinned bit-exact to the same
goldens by tests/test_oracle.py).

Bar: bit-exact (0 ulp) for the assembled MPI, its packed-layout form, the gradient
w.r.t. the network output, and the fused assemble+render path."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD, assert_bits

pytestmark = pytest.mark.gpu

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib, configs  # noqa: E402
from oracle import oracle  # noqa: E402

CASES = ("na", "nb", "nc")


@pytest.fixture(scope="module")
def net():
    return np.load(os.path.join(GOLD, "netout.npz"))


def _dep(net, c, dev):
    P = int(net[c + "_P"])
    B = net[c + "_pred"].shape[0]
    return {"mpi_planes": torch.zeros((B, P), device=dev), "ref_img": torch.tensor(net[c + "_ref"]).to(dev)}


@pytest.mark.parametrize("c", CASES)
def test_assemble_forward_vs_notebook(net, dev, c):
    pred = torch.tensor(net[c + "_pred"]).to(dev)
    rgba = mv.mpi_from_net_output(pred, _dep(net, c, dev))
    torch.cuda.synchronize()
    assert_bits(rgba.cpu().numpy(), net[c + "_rgba"], f"assembled MPI {c}")


@pytest.mark.parametrize("c", CASES)
def test_assemble_backward_vs_notebook_autograd(net, dev, c):
    pred = torch.tensor(net[c + "_pred"]).to(dev).requires_grad_(True)
    rgba = mv.mpi_from_net_output(pred, _dep(net, c, dev))
    rgba.backward(torch.tensor(net[c + "_drgba"]).to(dev))
    torch.cuda.synchronize()
    assert_bits(pred.grad.cpu().numpy(), net[c + "_dpred"], f"d pred {c}")


@pytest.mark.parametrize("c", CASES)
def test_assemble_backward_ref_image_vs_notebook_autograd(net, dev, c):
    """ref_img requiring grad too: d ref and d pred bit-exact to the notebook's
    autograd (which accumulates the per-plane g*w terms from the last plane to the first)."""
    pred = torch.tensor(net[c + "_pred"]).to(dev).requires_grad_(True)
    dep = _dep(net, c, dev)
    dep["ref_img"].requires_grad_(True)
    mv.mpi_from_net_output(pred, dep).backward(torch.tensor(net[c + "_drgba"]).to(dev))
    torch.cuda.synchronize()
    assert_bits(dep["ref_img"].grad.cpu().numpy(), net[c + "_dref"], f"d ref {c}")
    assert_bits(pred.grad.cpu().numpy(), net[c + "_dpred"], f"d pred {c}")


def test_backward_is_once_differentiable(dev):
    """Double backward through the HIP nodes raises instead of returning a graph-less
    gradient."""
    g = torch.Generator().manual_seed(3)
    B, H, W, P = 1, 12, 16, 4
    pred = (torch.rand((B, 2 * P + 3, H, W), generator=g) * 2 - 1).to(dev).requires_grad_(True)
    dep = {"mpi_planes": torch.zeros((B, P), device=dev), "ref_img": torch.rand((B, H, W, 3)).to(dev)}
    rgba = mv.mpi_from_net_output(pred, dep)
    (gp,) = torch.autograd.grad(rgba.sum(), pred, create_graph=True)
    with pytest.raises(RuntimeError):
        gp.sum().backward()


def test_assemble_strided_inputs(dev):
    """Non-contiguous prediction (a channels-last buffer viewed as NCHW) and reference
    image (a slice of a wider buffer): same bits as the oracle on dense copies."""
    g = torch.Generator().manual_seed(5)
    B, H, W, P = 2, 21, 34, 7
    nhwc = torch.rand((B, H, W, 2 * P + 3), generator=g) * 2 - 1
    wide = torch.rand((B, H, W, 5), generator=g) * 2 - 1
    pred = nhwc.to(dev).permute(0, 3, 1, 2)
    fg = wide.to(dev)[..., 1:4]
    rgba = _lib.assemble_mpi(pred, fg, P)
    drgba = torch.rand((B, H, W, P, 4), generator=g) * 2 - 1
    dpred = _lib.assemble_mpi_backward(drgba.to(dev), pred, fg, P)
    # a non-dense upstream gradient takes the generic (per-lane run) backward kernel
    dwide = torch.rand((B, H, W, P + 2, 4), generator=g) * 2 - 1
    dpred_s, dfg_s = _lib.assemble_mpi_backward(dwide.to(dev)[:, :, :, 1:P + 1], pred, fg, P, want_dfg=True)
    torch.cuda.synchronize()
    pn, fn = nhwc.permute(0, 3, 1, 2).contiguous().numpy(), wide[..., 1:4].contiguous().numpy()
    assert_bits(rgba.cpu().numpy(), oracle.assemble_mpi(pn, fn, P), "strided forward")
    assert_bits(dpred.cpu().numpy(), oracle.assemble_mpi_backward(drgba.numpy(), pn, fn, P), "dense backward")
    assert_bits(dpred_s.cpu().numpy(), oracle.assemble_mpi_backward(dwide[:, :, :, 1:P + 1].contiguous().numpy(),
                                                                    pn, fn, P), "strided backward")
    assert_bits(dfg_s.cpu().numpy(), oracle.assemble_mpi_backward_fg(dwide[:, :, :, 1:P + 1].contiguous().numpy(),
                                                                     pn, P), "strided backward d fg")


def test_assemble_packed_equals_pack_of_assembled(net, dev):
    pred = torch.tensor(net["nb_pred"]).to(dev)
    fg = torch.tensor(net["nb_ref"]).to(dev)
    P = int(net["nb_P"])
    packed = _lib.assemble_mpi_packed(pred, fg, P, 0)
    want = _lib.pack_planes(torch.tensor(net["nb_rgba"][0]).to(dev))
    torch.cuda.synchronize()
    assert_bits(packed.cpu().numpy(), want.cpu().numpy(), "assemble -> packed layout (incl. zero border)")


def test_fused_net_output_render(dev):
    """mpi_render_net_output_torch == mpi_render_view_torch(mpi_from_net_output(...)),
    bit for bit (B = 3 views, each with its own MPI)."""
    g = torch.Generator().manual_seed(9)
    B, H, W, P = 3, 40, 56, 8
    pred = (torch.rand((B, 2 * P + 3, H, W), generator=g) * 2 - 1).to(dev)
    ref = (torch.rand((B, H, W, 3), generator=g) * 2 - 1).to(dev)
    K = configs.f32([configs.intrinsics_matrix(50.0, 52.0, 28.0, 20.0)] * B).to(dev)
    poses = configs.f32([configs.pose_from(configs.rot_y(1.5 * (i - 1)), (0.03 * i, -0.02, 0.04))
                         for i in range(B)]).to(dev)
    planes = configs.f32(mv.inv_depths(1, 100, P)).to(dev)
    dep = {"mpi_planes": torch.zeros((B, P), device=dev), "ref_img": ref}
    want = mv.mpi_render_view_torch(mv.mpi_from_net_output(pred, dep), poses, planes, K)
    got = mv.mpi_render_net_output_torch(pred, ref, poses, planes, K)
    torch.cuda.synchronize()
    assert_bits(got.cpu().numpy(), want.cpu().numpy(), "fused assemble + render")


@pytest.mark.parametrize("geo", [0, 811, 821, 822, 422, 1821, -811, -821, -1821])
@pytest.mark.parametrize("case", ["odd", "extreme", "strided", "big"])
def test_fused_net_output_render_cases(case, geo, dev, kopts):
    """The one-kernel assembly + render (render_netout_kernel) against the two-step drop-ins
    (bit-exact, themselves pinned to the notebook / reference goldens): partial tiles, views
    with planes behind the camera (taps assembled directly, boxes that do not fit), a
    channel-strided prediction (a slice of a wider tensor) and a config-2-sized MPI."""
    g = torch.Generator().manual_seed(len(case))
    B, H, W, P = {"odd": (2, 37, 203, 7), "extreme": (4, 45, 70, 9), "strided": (2, 33, 64, 5),
                  "big": (1, 576, 1024, 32)}[case]
    pred = torch.rand((B, 2 * P + 3 + (4 if case == "strided" else 0), H, W), generator=g) * 2 - 1
    if case == "strided":
        pred = pred.to(dev)[:, 2:2 + 2 * P + 3]
        assert not pred.is_contiguous()
    else:
        pred = pred.to(dev)
    ref = (torch.rand((B, H, W, 3), generator=g) * 2 - 1).to(dev)
    f = configs.focal_from_fov(W)
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * B).to(dev)
    if case == "extreme":
        poses = [configs.pose_from(configs.rot_y((i - 1.5) * 25.0), ((i - 1.5) * 0.6, 0.3, (i - 2) * 0.7))
                 for i in range(B)]
    else:
        poses = [configs.pose_from(configs.rot_y(1.5 * (i - 1)), (0.03 * i, -0.02, 0.04)) for i in range(B)]
    poses = configs.f32(poses).to(dev)
    planes = configs.f32(mv.inv_depths(0.5 if case == "extreme" else 1, 100, P)).to(dev)
    dep = {"mpi_planes": torch.zeros((B, P), device=dev), "ref_img": ref}
    want = mv.mpi_render_view_torch(mv.mpi_from_net_output(pred, dep), poses, planes, K)
    # 0: automatic; 100 * waves + 10 * rows per work-item + planes in flight; negative: pointer loads
    kopts(netout_geo=abs(geo), netout_buf=0 if geo < 0 else 1)
    got = mv.mpi_render_net_output_torch(pred, ref, poses, planes, K)
    torch.cuda.synchronize()
    assert_bits(got.cpu().numpy(), want.cpu().numpy(), f"fused assemble + render ({case}, geo {geo})")


NETOUT_TRAIN = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "netout_train.npz"))


@pytest.mark.parametrize("case", ["ta", "tb", "tc", "td"])
@pytest.mark.parametrize("wants", ["both", "pred", "ref"])
def test_fused_net_output_training_vs_reference(case, wants, dev):
    """Training through the fused net-output render (the notebook's losses, ipynb cell 12 L7-11 /
    L38-42: mpi_from_net_output then mpi_render_view_torch): frames, d network output and d
    reference image bit-exact vs the reference's CPU autograd (tests/golden/netout_train.npz:
    8, 12, 17 and 32 planes -- one, two and several checkpoint chunks)."""
    g = NETOUT_TRAIN
    pred = torch.tensor(g[case + "_pred"]).to(dev).requires_grad_(wants in ("both", "pred"))
    ref = torch.tensor(g[case + "_ref"]).to(dev).requires_grad_(wants in ("both", "ref"))
    pose, K, depths = (torch.tensor(g[f"{case}_{k}"]).to(dev) for k in ("pose", "K", "depths"))
    out = mv.mpi_render_net_output_torch(pred, ref, pose, depths, K)
    assert out.grad_fn is not None and "NetOutputRender" in type(out.grad_fn).__name__
    out.backward(torch.tensor(g[case + "_dout"]).to(dev))
    torch.cuda.synchronize()
    assert_bits(out.detach().cpu().numpy(), g[case + "_out"], f"frames {case}")
    if wants != "ref":
        assert_bits(pred.grad.cpu().numpy(), g[case + "_dpred"], f"d pred {case}")
    if wants != "pred":
        assert_bits(ref.grad.cpu().numpy(), g[case + "_dref"], f"d ref_img {case}")


@pytest.mark.parametrize("buf", [1, 0])
@pytest.mark.parametrize("shape", [(2, 24, 40, 12), (1, 33, 47, 17), (1, 40, 64, 8), (1, 576, 1024, 32),
                                   (2, 45, 70, 9)])
def test_netout_train_checkpoints_equal_render_train(shape, buf, dev, kopts):
    """The fused training forward's composite checkpoints equal mpiv_render_train's for the
    assembled MPI (slots 1.. -- slot 0 is never written or read), and its frames the inference
    kernel's, bit for bit; incl. a view with planes behind the camera (taps assembled directly)."""
    B, H, W, P = shape
    gen = torch.Generator().manual_seed(H * W + P)
    pred = (torch.rand((B, 2 * P + 3, H, W), generator=gen) * 2 - 1).to(dev)
    ref = (torch.rand((B, H, W, 3), generator=gen) * 2 - 1).to(dev)
    f = configs.focal_from_fov(W)
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * B)
    big = W == 70
    poses = configs.f32([configs.pose_from(configs.rot_y((i + 1) * (20.0 if big else 1.2)),
                                           ((i + 1) * (0.5 if big else 0.03), -0.02, 0.04 - (0.6 if big else 0)))
                         for i in range(B)])
    homs = _host.render_homographies(poses, configs.f32(mv.inv_depths(0.5 if big else 1, 100, P)), K, B).to(dev)
    kopts(netout_buf=buf)
    out, ck = _lib.render_net_output_train(pred, ref, P, homs)
    inf = _lib.render_net_output(pred, ref, P, homs)
    f2, ck2 = _lib.render_train(_lib.assemble_mpi(pred, ref, P), homs)
    torch.cuda.synchronize()
    assert ck is not None and ck2 is not None and ck.shape == ck2.shape
    assert_bits(out.cpu().numpy(), inf.cpu().numpy(), "train forward frames vs inference kernel")
    assert_bits(out.cpu().numpy(), f2.cpu().numpy(), "train forward frames vs two-step")
    assert_bits(ck[:, 1:].cpu().numpy(), ck2[:, 1:].cpu().numpy(), "checkpoints vs render_train")


def test_fused_net_output_training_equals_two_step_at_config2_size(dev):
    """At config 2's size (1024x576, 32 planes) the fused training step gives the two-step
    chain's gradients (mpi_from_net_output -> mpi_render_view_torch under autograd) bit for bit."""
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    gen = torch.Generator().manual_seed(12)
    pred0 = (torch.rand((1, 2 * P + 3, H, W), generator=gen) * 2 - 1).to(dev)
    ref0 = (torch.rand((1, H, W, 3), generator=gen) * 2 - 1).to(dev)
    dout = (torch.rand((1, H, W, 3), generator=gen) * 2 - 1).to(dev)
    pose = configs.f32(c["poses"][7:8]).to(dev)
    K = configs.f32([c["K"]]).to(dev)
    planes = configs.f32(c["depths"]).to(dev)
    p1, r1 = pred0.clone().requires_grad_(True), ref0.clone().requires_grad_(True)
    mv.mpi_render_net_output_torch(p1, r1, pose, planes, K).backward(dout)
    p2, r2 = pred0.clone().requires_grad_(True), ref0.clone().requires_grad_(True)
    dep = {"mpi_planes": torch.zeros((1, P), device=dev), "ref_img": r2}
    mv.mpi_render_view_torch(mv.mpi_from_net_output(p2, dep), pose, planes, K).backward(dout)
    torch.cuda.synchronize()
    assert_bits(p1.grad.cpu().numpy(), p2.grad.cpu().numpy(), "d pred fused vs two-step")
    assert_bits(r1.grad.cpu().numpy(), r2.grad.cpu().numpy(), "d ref_img fused vs two-step")


def test_fused_net_output_training_strided_and_partial_grads(dev):
    """Training through the fused render with a channel-strided network output (a slice of a wider
    tensor, as a network head's output view can be) and a B = 3 batch of different MPIs: d pred and
    d ref_img equal the two-step chain's bit for bit; a second backward through a new graph reuses nothing
    stale."""
    gen = torch.Generator().manual_seed(77)
    B, H, W, P = 3, 29, 45, 11
    wide = (torch.rand((B, 2 * P + 3 + 5, H, W), generator=gen) * 2 - 1).to(dev)
    ref0 = (torch.rand((B, H, W, 3), generator=gen) * 2 - 1).to(dev)
    dout = (torch.rand((B, H, W, 3), generator=gen) * 2 - 1).to(dev)
    f = configs.focal_from_fov(W)
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * B).to(dev)
    poses = configs.f32([configs.pose_from(configs.rot_y(2.0 * (i - 1)), (0.04 * i, -0.02, 0.05)) for i in range(B)]).to(dev)
    planes = configs.f32(mv.inv_depths(1, 60, P)).to(dev)
    grads = []
    for fused in (True, False):
        w = wide.clone().requires_grad_(True)
        pred = w[:, 3:3 + 2 * P + 3]
        assert not pred.is_contiguous()
        ref = ref0.clone().requires_grad_(True)
        if fused:
            out = mv.mpi_render_net_output_torch(pred, ref, poses, planes, K)
        else:
            dep = {"mpi_planes": torch.zeros((B, P), device=dev), "ref_img": ref}
            out = mv.mpi_render_view_torch(mv.mpi_from_net_output(pred, dep), poses, planes, K)
        out.backward(dout)
        torch.cuda.synchronize()
        grads.append((w.grad.cpu().numpy(), ref.grad.cpu().numpy(), out.detach().cpu().numpy()))
    assert_bits(grads[0][2], grads[1][2], "frames")
    assert_bits(grads[0][0], grads[1][0], "d network output (strided slice)")
    assert_bits(grads[0][1], grads[1][1], "d ref_img")


@pytest.mark.parametrize("shape", [(54, 230, 12), (48, 80, 20), (72, 72, 9), (33, 47, 17)])
def test_assemble_sampled_rows_cover_every_read(shape, dev):
    """mpiv_assemble_mpi_sampled (the fused training's re-assembly, round 6) leaves the texel rows no
    output pixel samples unwritten: with those rows NaN-filled, the render and its backward equal the
    ones over the whole assembly bit for bit (a NaN read anywhere would show), the written texels equal
    mpiv_assemble_mpi's, and on a landscape MPI (the swapped normalisation samples its top rows only)
    texels are actually skipped.  Camera-path, rotated and extreme poses (planes behind the camera:
    bounds not provable, every row written)."""
    H, W, P = shape
    g = torch.Generator().manual_seed(H * W + P)
    pred = (torch.rand((3, 2 * P + 3, H, W), generator=g) * 2 - 1).to(dev)
    fg = (torch.rand((3, H, W, 3), generator=g) * 2 - 1).to(dev)
    f = configs.focal_from_fov(W)
    K = configs.f32([configs.intrinsics_matrix(f, f, W / 2.0, H / 2.0)] * 3)
    poses = configs.f32([configs.sway_path(1000)[250],
                         configs.pose_from(configs.rot_y(11.0), (0.3, -0.15, 0.25)),
                         configs.pose_from(configs.rot_y(-40.0), (1.5, 0.4, -2.0))])
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(0.5, 50, P)), K, 3).to(dev)
    full = _lib.assemble_mpi(pred, fg, P)
    part = torch.full_like(full, float("nan"))
    _lib._call("mpiv_assemble_mpi_sampled", pred, _lib._strides(pred), fg, _lib._strides(fg), 3, H, W, P, homs, part,
               _lib._stream(dev))
    torch.cuda.synchronize()
    written = ~torch.isnan(part).any(dim=-1)  # [B, H, W, P]: blocks of 64 pixels x 16 planes are skipped whole
    assert torch.equal(part[written].view(torch.int32), full[written].view(torch.int32))
    if W > H:
        assert not bool(written[0].all()), "a landscape MPI's unsampled rows are skipped"
    dout = (torch.rand((3, H, W, 3), generator=g) * 2 - 1).to(dev)
    assert_bits(_lib.render(part, homs).cpu().numpy(), _lib.render(full, homs).cpu().numpy(), "render")
    want = _lib.render_backward(full, homs, dout, check=True)
    assert_bits(_lib.render_backward(part, homs, dout, check=True).cpu().numpy(), want.cpu().numpy(), "backward")
    _, ck = _lib.render_train(full, homs)
    assert_bits(_lib.render_backward(part, homs, dout, ckpt=ck, check=True).cpu().numpy(), want.cpu().numpy(),
                "backward with checkpoints")

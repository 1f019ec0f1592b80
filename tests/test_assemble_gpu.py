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
from mpi_vision_amd import _lib, configs  # noqa: E402
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

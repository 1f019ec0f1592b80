"""The PSV's intrinsics layout: the reference inverts the caller's
intrinsics tensor as passed (`torch.inverse(intrinsics)`, utils.py:370, reached from :428 and
:747), and torch's CPU inverse gives other bits for the same values in another layout -- a
shared camera as K[None].expand(B,3,3) (stride 0), F-ordered or sliced blocks, a transposed
unbatched K for the `_one` call.  tests/golden/kstride.npz holds the reference's own outputs
for those layouts (tools/gen_goldens_kstride.py; each case is one whose layout moves the
reference's output, by up to 8.5e-5).

torch's CPU inverse is also HOST-dependent (MKL dispatch: on the AMD EPYC GPU box 3 of these
cameras invert 1 ulp differently from the Intel host that ran the reference, in either layout), so
the goldens also record the reference's K^-1 bits (`<case>_ki`):
CPU: the oracle with the reference's K^-1 reproduces every golden (host-independent); the drop-in's
     K^-1 is torch.inverse of the caller's layout on this host (= the recorded bits on the golden host).
GPU: the kernels with the reference's K^-1 reproduce the goldens; the drop-in (host pose and HBM pose
     paths) equals the oracle fed with this host's reference computation, and the golden wherever
     the host's LAPACK agrees."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD, assert_bits

import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib  # noqa: E402
from oracle import oracle  # noqa: E402

PSV_CASES = ["psv_expand", "psv_fortran", "psv_slice"]


@pytest.fixture(scope="module")
def ks():
    return np.load(os.path.join(GOLD, "kstride.npz"))


def make_layout(K: torch.Tensor, layout: str) -> torch.Tensor:
    """The caller's tensor with K's values (same helper as tools/gen_goldens_kstride.py);
    built on K's device, so a device K keeps the layout too."""
    if layout == "expand":
        return K[:1].expand(K.shape[0], 3, 3)
    if layout == "fortran":
        return K.transpose(1, 2).contiguous().transpose(1, 2)
    if layout == "slice":
        buf = torch.zeros(K.shape[0], 3, 5, device=K.device)
        buf[:, :, :3] = K
        return buf[:, :, :3]
    if layout == "t1":
        return K[0].t().contiguous().t()
    raise ValueError(layout)


def _case(ks, c, dev=None):
    t = {k[len(c) + 1:]: ks[k] for k in ks.files if k.startswith(c + "_")}
    layout = str(t.pop("layout"))
    conv = {k: (torch.tensor(v) if v.dtype != object and v.dtype.kind == "f" else v) for k, v in t.items()}
    if dev is not None:
        conv = {k: (v.to(dev) if isinstance(v, torch.Tensor) else v) for k, v in conv.items()}
    return conv, layout


def test_layouts_are_what_the_goldens_say(ks):
    """The rebuilt caller tensors really have the layouts the goldens were made with."""
    K = torch.tensor(ks["psv_expand_K"])
    assert make_layout(K, "expand").stride(0) == 0
    assert make_layout(K, "fortran").stride()[1:] == (1, 3)
    assert make_layout(K, "slice").stride() == (15, 5, 1)
    assert make_layout(torch.tensor(ks["one_t1_K"]), "t1").stride() == (1, 3)


def _host_mats(t, layout, tgt_key="K"):
    """This host's drop-in matrices for the case: Ki = torch.inverse of the caller's layout
    (psv_inverse), proj = K4_src @ pose."""
    pose = t["pose"] if t["pose"].dim() == 3 else t["pose"][None]
    Ks = make_layout(t["K"].cpu(), layout)
    Kt = make_layout(t[tgt_key].cpu(), layout)
    if layout == "t1":  # plane_sweep_torch_one's unsqueeze (utils.py:530)
        Ks, Kt = Ks.unsqueeze(0), Kt.unsqueeze(0)
    return _host.psv_matrices(Ks, Kt, pose.cpu())


def _sweep_oracle(t, ki, proj):
    img = t["img"].cpu()
    img = img if img.dim() == 4 else img[None]
    return oracle.plane_sweep(img.numpy(), np.ascontiguousarray(ki, np.float32).reshape(-1, 9), proj.numpy(),
                              [float(d) for d in t["depths"]], img.shape[1], img.shape[2])


@pytest.mark.parametrize("c", PSV_CASES + ["one_t1"])
def test_oracle_with_reference_inverse_equals_golden(ks, c):
    """The rest of the chain, pinned host-independently: the reference's own K^-1 bits (recorded
    by the generator), this host's proj and the oracle reproduce the reference's volume."""
    t, layout = _case(ks, c)
    _, proj = _host_mats(t, layout)
    assert_bits(_sweep_oracle(t, ks[c + "_ki"], proj), ks[c + "_out"], c)


def test_oracle_warps_with_reference_inverse(ks):
    for c, tk in (("piw_expand", "K"), ("piw2_expand", "Kt")):
        t, layout = _case(ks, c)
        _, proj = _host_mats(t, layout, tk)
        ki = np.ascontiguousarray(ks[c + "_ki"]).reshape(-1, 9)
        assert_bits(oracle.inverse_warp(t["img"].numpy(), ki, proj.numpy(), t["depth"].numpy()), ks[c + "_out"], c)


@pytest.mark.parametrize("c", PSV_CASES + ["one_t1", "piw_expand", "piw2_expand"])
def test_drop_in_inverts_the_callers_layout(ks, c):
    """psv_matrices' Ki is torch.inverse of the caller's tensor AS LAID OUT on this host (what
    pixel2cam_torch computes, utils.py:370) -- not of a materialised copy; on the host that made
    the goldens that is the reference's recorded inverse.  (MKL's inverse is host-dependent: on an
    AMD EPYC box 3 of these cameras invert 1 ulp differently in either layout,
    tools/probes/inverse_layouts.py; the drop-in then matches the reference run on that host.)"""
    t, layout = _case(ks, c)
    tk = "Kt" if c == "piw2_expand" else "K"
    ki, _ = _host_mats(t, layout, tk)
    Kl = make_layout(t[tk], layout)
    if layout == "t1":
        Kl = Kl.unsqueeze(0)
    own = torch.inverse(Kl).contiguous().reshape(ki.shape)
    assert_bits(ki, own, c)
    if np.array_equal(own.numpy().view(np.uint32), np.ascontiguousarray(ks[c + "_ki"]).reshape(ki.shape).view(np.uint32)):
        Kc = t[tk].unsqueeze(0) if layout == "t1" else t[tk]
        assert not torch.equal(own, torch.inverse(Kc.contiguous()).reshape(ki.shape)), \
            f"{c}: this camera inverts layout-independently here: the golden pins nothing"


def test_cpu32_like_keeps_strides():
    K = torch.arange(9, dtype=torch.float64).reshape(1, 3, 3).expand(4, 3, 3)
    c = _host.cpu32_like(K)
    assert c.dtype == torch.float32 and c.stride() == K.stride() and torch.equal(c, K.float())
    buf = torch.arange(60, dtype=torch.float32).reshape(4, 3, 5)[1:, :, 1:4]
    c = _host.cpu32_like(buf.double())  # dtype conversion materialises: values survive
    assert torch.equal(c, buf)


def _golden_if_host_agrees(ks, c, ki):
    """The reference's own output is the golden only where this host's inverse equals the
    reference host's (see test_drop_in_inverts_the_callers_layout)."""
    return np.array_equal(np.ascontiguousarray(ki.cpu().numpy(), np.float32).reshape(-1).view(np.uint32),
                          np.ascontiguousarray(ks[c + "_ki"], np.float32).reshape(-1).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("pose_on_dev", [False, True])
@pytest.mark.parametrize("c", PSV_CASES)
def test_drop_in_psv_caller_layout(ks, c, pose_on_dev, dev):
    """plane_sweep_torch with the caller's K layout on the device, host-pose path (psv_matrices)
    and HBM-pose path (psv_ki_device + device proj): bit-exact to the oracle fed with the
    reference's computation on this host (K^-1 of the caller's layout), and to the reference's
    golden wherever this host's LAPACK agrees with the golden host's."""
    t, layout = _case(ks, c, dev)
    Kl = make_layout(t["K"], layout)
    assert Kl.is_cuda and Kl.stride() == make_layout(t["K"].cpu(), layout).stride()
    pose = t["pose"] if pose_on_dev else t["pose"].cpu()
    ki, proj = _host_mats(t, layout)
    want = _sweep_oracle(t, ki.numpy(), proj)
    for _ in range(2):  # second call through the memoised inverse
        out = mv.plane_sweep_torch(t["img"], [float(d) for d in t["depths"]], pose, Kl)
        assert_bits(out, want, f"{c} pose_on_dev={pose_on_dev}")
    if _golden_if_host_agrees(ks, c, ki):
        assert_bits(out, ks[c + "_out"], f"{c} vs reference golden")


@pytest.mark.gpu
@pytest.mark.parametrize("c", PSV_CASES + ["one_t1"])
def test_kernel_with_reference_inverse_equals_golden(ks, c, dev):
    """The HIP sweep given the reference's recorded K^-1: the reference's volume, on any host."""
    t, layout = _case(ks, c)
    _, proj = _host_mats(t, layout)
    img = t["img"] if t["img"].dim() == 4 else t["img"][None]
    ki = torch.tensor(np.ascontiguousarray(ks[c + "_ki"]).reshape(-1, 9)).to(dev)
    out = _lib.plane_sweep(img.to(dev), [float(d) for d in t["depths"]], ki, proj.to(dev), img.shape[1], img.shape[2])
    assert_bits(out, ks[c + "_out"], c)


@pytest.mark.gpu
@pytest.mark.parametrize("pose_on_dev", [False, True])
def test_drop_in_warps_caller_layout(ks, pose_on_dev, dev):
    for c, tk in (("piw_expand", "K"), ("piw2_expand", "Kt")):
        t, layout = _case(ks, c, dev)
        pose = t["pose"] if pose_on_dev else t["pose"].cpu()
        ki, proj = _host_mats(t, layout, tk)
        want = oracle.inverse_warp(t["img"].cpu().numpy(), ki.numpy(), proj.numpy(), t["depth"].cpu().numpy())
        if c == "piw_expand":
            out = mv.projective_inverse_warp_torch(t["img"], t["depth"], pose, make_layout(t["K"], layout))
        else:
            Ht, Wt = (int(v) for v in ks["piw2_expand_tgt"])
            out = mv.projective_inverse_warp_torch2(t["img"], t["depth"], pose, make_layout(t["K"], layout),
                                                    make_layout(t["Kt"], layout), Ht, Wt)
        assert_bits(out, want, c)
        if _golden_if_host_agrees(ks, c, ki):
            assert_bits(out, ks[c + "_out"], f"{c} vs reference golden")
        ki_ref = torch.tensor(np.ascontiguousarray(ks[c + "_ki"]).reshape(-1, 9)).to(dev)
        assert_bits(_lib.inverse_warp_depthmap(t["img"], t["depth"], ki_ref, proj.to(dev), *out.shape[1:3]),
                    ks[c + "_out"], c + " with the reference's inverse")


@pytest.mark.gpu
@pytest.mark.parametrize("pose_on_dev", [False, True])
def test_drop_in_one_transposed_camera(ks, pose_on_dev, dev):
    t, layout = _case(ks, "one_t1", dev)
    pose = t["pose"] if pose_on_dev else t["pose"].cpu()
    ki, proj = _host_mats(t, layout)
    out = mv.plane_sweep_torch_one(t["img"], [float(d) for d in t["depths"]], pose, make_layout(t["K"], layout))
    assert_bits(out, _sweep_oracle(t, ki.numpy(), proj), "one_t1")
    if _golden_if_host_agrees(ks, "one_t1", ki):
        assert_bits(out, ks["one_t1_out"], "one_t1 vs reference golden")


@pytest.mark.gpu
def test_render_and_psv_memo_do_not_mix(ks, dev):
    """One intrinsics tensor used by the render (materialised inverse, utils.py:225-228) and by
    the PSV (caller's layout) keeps two memo entries: each path gets its own bits."""
    t, layout = _case(ks, "psv_expand", dev)
    Kl = make_layout(t["K"], layout)
    B = Kl.shape[0]
    r = _host._kinv_device(Kl, B, dev)
    p = _host.psv_ki_device(Kl, B, dev)
    assert_bits(r, torch.inverse(t["K"].cpu().contiguous()), "render inverse")
    assert_bits(p, torch.inverse(make_layout(t["K"].cpu(), layout)), "psv inverse")

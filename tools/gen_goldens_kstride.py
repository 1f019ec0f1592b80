#!/usr/bin/env python3
"""Golden fixtures for the PSV's intrinsics STRIDE PATTERN.

The reference inverts the caller's intrinsics tensor as passed: `torch.inverse(intrinsics)`
in pixel2cam_torch (utils.py:370, reached from projective_inverse_warp_torch :428 and
projective_inverse_warp_torch2 :747).  torch's CPU inverse returns different bits for the
same 3x3 values laid out differently -- a stride-0 batch (`K[None].expand(B,3,3)`, the usual
way to share one camera), Fortran-ordered blocks, a slice of a wider buffer -- and the PSV
moves by up to ~5e-5 with it.  This script runs the REFERENCE utils.py on CPU (the import
recipe of tools/gen_goldens.py) on such layouts and writes tests/golden/kstride.npz:

    <case>_img, <case>_pose, <case>_K (values, contiguous), <case>_layout (str),
    <case>_depths (PSV) | <case>_depth (depth-map warps), <case>_out,
    <case>_Kt / <case>_tgt for the _2 cases,
    <case>_ki: torch.inverse of the caller's (target) intrinsics tensor as the reference computed it
    on THIS host -- MKL's CPU inverse is host-dependent (an AMD EPYC box returns 1-ulp-different
    bits for 3 of these cameras, in both layouts), so the tests pin the rest of the chain with
    these bits and compare the host's own inverse to them only where the host agrees

`layout` names how the test rebuilds the caller's tensor from K's values (tests/test_kstride.py
`make_layout`): "expand" = K[:1].expand(B,3,3), "fortran" = F-ordered [B,3,3] blocks,
"slice" = [:, :, :3] of a [B,3,5] buffer, "t1" = an unbatched [3,3] given transposed
(K.t().contiguous().t()).  Each case also asserts the layout changes the reference's own
output, so the goldens pin something the contiguous goldens do not.

Usage:  python tools/gen_goldens_kstride.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from gen_goldens import f32, load_reference, rand_pose  # noqa: E402
from mpi_vision_amd import configs  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "kstride.npz")


def make_layout(K: torch.Tensor, layout: str) -> torch.Tensor:
    """Same helper as tests/test_kstride.py: the caller's tensor with K's values."""
    if layout == "expand":
        return K[:1].expand(K.shape[0], 3, 3)
    if layout == "fortran":
        return K.transpose(1, 2).contiguous().transpose(1, 2)
    if layout == "slice":
        buf = torch.zeros(K.shape[0], 3, 5)
        buf[:, :, :3] = K
        return buf[:, :, :3]
    if layout == "t1":
        return K[0].t().contiguous().t()
    raise ValueError(layout)


def rand_K(g, B):
    return f32([configs.intrinsics_matrix(*(torch.rand(4, generator=g) * 300 + 5).tolist()) for _ in range(B)])


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    g = torch.Generator().manual_seed(505)
    out = {}

    def keep(tag, **kv):
        for k, v in kv.items():
            out[f"{tag}_{k}"] = v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)

    # plane_sweep_torch (utils.py:452-471): B = 4 views sharing one camera, 3 layouts
    B, H, W, D = 4, 48, 64, 12
    depths = configs.inv_depths(1, 100, D)
    for layout in ("expand", "fortran", "slice"):
        img = torch.rand((B, H, W, 3), generator=g)
        pose = f32([rand_pose(g, 0.1, 0.3) for _ in range(B)])
        for _ in range(64):  # a camera whose layout moves the reference's output
            K = rand_K(g, 1).expand(B, 3, 3).contiguous() if layout == "expand" else rand_K(g, B)
            got = ref.plane_sweep_torch(img, depths, pose, make_layout(K, layout))
            diff = float((got - ref.plane_sweep_torch(img, depths, pose, K)).abs().max())
            if diff > 0:
                break
        else:
            raise AssertionError(f"psv_{layout}: no camera found whose layout changes the output")
        print(f"psv_{layout}: layout moves the reference output by up to {diff:.3g}")
        keep(f"psv_{layout}", img=img, pose=pose, K=K, layout=layout, depths=np.array(depths), out=got,
             ki=torch.inverse(make_layout(K, layout)).contiguous())

    # projective_inverse_warp_torch (utils.py:409-450) with a depth map, shared camera
    B, H, W = 3, 30, 44
    img = torch.rand((B, H, W, 3), generator=g)
    depth = torch.rand((B, H, W), generator=g) * 30 + 0.5
    pose = f32([rand_pose(g, 0.1, 0.4) for _ in range(B)])
    for _ in range(64):
        K = rand_K(g, 1).expand(B, 3, 3).contiguous()
        got = ref.projective_inverse_warp_torch(img, depth, pose, make_layout(K, "expand"))
        if float((got - ref.projective_inverse_warp_torch(img, depth, pose, K)).abs().max()) > 0:
            break
    else:
        raise AssertionError("piw_expand: no camera found whose layout changes the output")
    keep("piw_expand", img=img, depth=depth, pose=pose, K=K, layout="expand", out=got,
         ki=torch.inverse(make_layout(K, "expand")).contiguous())

    # projective_inverse_warp_torch2 (utils.py:725-769): shared source AND target cameras
    B, Hs, Ws, Ht, Wt = 2, 36, 48, 28, 70
    img = torch.rand((B, Hs, Ws, 3), generator=g)
    depth = torch.rand((B, Ht, Wt), generator=g) * 20 + 0.5
    pose = f32([rand_pose(g, 0.08, 0.3) for _ in range(B)])
    Ks = rand_K(g, 1).expand(B, 3, 3).contiguous()
    for _ in range(64):
        Kt = rand_K(g, 1).expand(B, 3, 3).contiguous()
        got = ref.projective_inverse_warp_torch2(img, depth, pose, make_layout(Ks, "expand"),
                                                 make_layout(Kt, "expand"), Ht, Wt)
        if float((got - ref.projective_inverse_warp_torch2(img, depth, pose, Ks, Kt, Ht, Wt)).abs().max()) > 0:
            break
    else:
        raise AssertionError("piw2_expand: no camera found whose layout changes the output")
    keep("piw2_expand", img=img, depth=depth, pose=pose, K=Ks, Kt=Kt, layout="expand", tgt=np.array([Ht, Wt]),
         out=got, ki=torch.inverse(make_layout(Kt, "expand")).contiguous())

    # plane_sweep_torch_one (utils.py:513-533): an unbatched camera given transposed
    H, W, D = 40, 56, 10
    img = torch.rand((H, W, 3), generator=g)
    pose = f32(rand_pose(g, 0.1, 0.3))
    depths = configs.inv_depths(1, 100, D)
    K = rand_K(g, 1)
    for _ in range(64):  # a camera whose transposed layout moves the reference's output
        got = ref.plane_sweep_torch_one(img, depths, pose, make_layout(K, "t1"))
        if float((got - ref.plane_sweep_torch_one(img, depths, pose, K[0])).abs().max()) > 0:
            break
        K = rand_K(g, 1)
    else:
        raise AssertionError("no camera found whose transposed layout changes the output")
    keep("one_t1", img=img, pose=pose, K=K, layout="t1", depths=np.array(depths), out=got,
         ki=torch.inverse(make_layout(K, "t1").unsqueeze(0)).contiguous())

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items() if k.endswith("_out")})


if __name__ == "__main__":
    main()

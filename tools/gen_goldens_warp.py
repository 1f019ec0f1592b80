#!/usr/bin/env python3
"""Golden fixtures for the depth-map inverse warps (SURVEY.md §8a rows
`projective_inverse_warp_torch` utils.py:409-450 and `projective_inverse_warp_torch2`
utils.py:725-769) with NON-constant depth maps -- the PSV goldens only exercise
constant-depth slices.  Runs the REFERENCE utils.py on CPU (the import recipe of
tools/gen_goldens.py); writes tests/golden/warp.npz:

    <case>_img, <case>_depth, <case>_pose, <case>_K[s|t], <case>_out   (+ tgt size for _2 cases)

Usage:  python tools/gen_goldens_warp.py
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

OUT = os.path.join(REPO, "tests", "golden", "warp.npz")


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    g = torch.Generator().manual_seed(77)
    out = {}

    # projective_inverse_warp_torch: B=2, 3-channel, a smooth depth ramp + noise, one
    # pixel at depth 0 (cam point at the origin: z + 1e-10 in cam2pixel) and some negative
    # depths (points behind the camera)
    B, H, W = 2, 30, 44
    img = torch.rand((B, H, W, 3), generator=g)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    depth = (1.0 + 0.2 * xx + 0.1 * yy).expand(B, H, W).clone() + torch.rand((B, H, W), generator=g) * 3
    depth[0, 0, 0] = 0.0
    depth[1, 5:8, 10:14] = -2.0
    K = f32([configs.intrinsics_matrix(40.0, 42.0, 22.0, 15.0), configs.intrinsics_matrix(38.0, 38.0, 21.0, 14.5)])
    pose = f32([rand_pose(g, 0.1, 0.4), rand_pose(g, 0.3, 1.0)])
    res = ref.projective_inverse_warp_torch(img, depth, pose, K)
    out.update(piw_img=img.numpy(), piw_depth=depth.numpy(), piw_pose=pose.numpy(), piw_K=K.numpy(),
               piw_out=res.numpy())

    # 4-channel source, B=1, strongly varying depth (near / far mix)
    img = torch.rand((1, 25, 25, 4), generator=g)
    depth = torch.where(torch.rand((1, 25, 25), generator=g) > 0.5, torch.tensor(0.7), torch.tensor(60.0))
    K = f32([configs.intrinsics_matrix(30.0, 30.0, 12.0, 12.0)])
    pose = f32([rand_pose(g, 0.05, 0.2)])
    res = ref.projective_inverse_warp_torch(img, depth, pose, K)
    out.update(piw4_img=img.numpy(), piw4_depth=depth.numpy(), piw4_pose=pose.numpy(), piw4_K=K.numpy(),
               piw4_out=res.numpy())

    # projective_inverse_warp_torch2: separate intrinsics, target grid != source size
    B, Hs, Ws, Ht, Wt = 2, 36, 48, 28, 70
    img = torch.rand((B, Hs, Ws, 3), generator=g)
    depth = torch.rand((B, Ht, Wt), generator=g) * 20 + 0.5
    Ks = f32([configs.intrinsics_matrix(45.0, 46.0, 24.0, 18.0), configs.intrinsics_matrix(50.0, 50.0, 23.0, 17.0)])
    Kt = f32([configs.intrinsics_matrix(60.0, 58.0, 35.0, 14.0), configs.intrinsics_matrix(55.0, 55.0, 34.0, 13.5)])
    pose = f32([rand_pose(g, 0.08, 0.3), rand_pose(g, 0.08, 0.3)])
    res = ref.projective_inverse_warp_torch2(img, depth, pose, Ks, Kt, Ht, Wt)
    out.update(piw2_img=img.numpy(), piw2_depth=depth.numpy(), piw2_pose=pose.numpy(), piw2_Ks=Ks.numpy(),
               piw2_Kt=Kt.numpy(), piw2_tgt=np.array([Ht, Wt]), piw2_out=res.numpy())
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items() if k.endswith("_out")})


if __name__ == "__main__":
    main()

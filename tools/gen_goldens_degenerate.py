#!/usr/bin/env python3
"""Goldens for degenerate frame sizes (H or W = 1, 2x2): the reference's
mpi_render_view_torch run on CPU (imported as in gen_goldens.py).  H = 1 or W = 1 makes
the reference divide by H-1 = 0 or W-1 = 0 (utils.py:188), so its output holds NaN where
it does; the drop-in must reproduce those bits.  Writes tests/golden/degenerate.npz."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
from gen_goldens import load_reference  # noqa: E402
from mpi_vision_amd import configs  # noqa: E402

CASES = [(1, 7, 3), (5, 1, 3), (2, 2, 2), (1, 1, 2)]


def main():
    ref = load_reference()
    out = {}
    for (H, W, P) in CASES:
        tag = f"h{H}w{W}p{P}"
        g = torch.Generator().manual_seed(H * 10 + W)
        mpi = torch.rand((1, H, W, P, 4), generator=g) * 2 - 1
        K = configs.f32([configs.intrinsics_matrix(5.0, 5.5, W / 2, H / 2)])
        pose = configs.f32([configs.pose_from(configs.rot_y(1.0), (0.05, -0.02, 0.03))])
        planes = configs.f32(configs.inv_depths(1, 10, P))
        out[tag + "_mpi"] = mpi.numpy()
        out[tag + "_K"] = K.numpy()
        out[tag + "_pose"] = pose.numpy()
        out[tag + "_planes"] = planes.numpy()
        out[tag + "_out"] = ref.mpi_render_view_torch(mpi, pose, planes, K).numpy()
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "degenerate.npz"), **out)


if __name__ == "__main__":
    main()

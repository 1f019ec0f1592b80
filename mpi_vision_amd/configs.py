"""Workload definitions for the BASELINE.json configs.

Camera models follow the reference's DeepView viewer template
(`deepview-mpi-viewer-template.html:304` focal = 0.5*W/tan(fov/2), defaults
near=1, far=100, fov=60 at `:674-676`) and the notebook's plane spacing
(`inv_depths(1, 100, P)`, `fast-torch-stereo-vision.ipynb` cell 8 L73).

Every pose / intrinsics value is produced with Python's `math` module in
float64 and rounded once to float32, so the same numbers come out on any x86
host (no SIMD libm in the path).  Golden fixtures also store the exact fp32
values they were generated with.
"""
from __future__ import annotations

import math

import torch

from .utils import inv_depths


def focal_from_fov(width: int, fov_deg: float = 60.0) -> float:
    """Viewer focal length in pixels (`deepview-mpi-viewer-template.html:304`)."""
    return 0.5 * width / math.tan(math.radians(fov_deg) / 2.0)


def rot_y(deg: float):
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    return [[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]]


def pose_from(R, t):
    """4x4 rigid transform p_t = R p_s + t as nested float64 lists."""
    return [[R[0][0], R[0][1], R[0][2], t[0]],
            [R[1][0], R[1][1], R[1][2], t[1]],
            [R[2][0], R[2][1], R[2][2], t[2]],
            [0.0, 0.0, 0.0, 1.0]]


def intrinsics_matrix(fx: float, fy: float, cx: float, cy: float):
    return [[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]]


def sway_path(n: int):
    """'sway/wander' camera path like the viewer's (`html:620-639`), SURVEY §8d C2/C4."""
    poses = []
    for k in range(n):
        a = 2.0 * math.pi * k / n
        t = (0.05 * math.sin(a), 0.02 * math.cos(a), 0.03 * math.sin(math.pi * k / n))
        poses.append(pose_from(rot_y(1.0 * math.sin(a)), t))
    return poses


def f32(x) -> torch.Tensor:
    return torch.tensor(x, dtype=torch.float64).to(torch.float32)


def synthetic_mpi(batch: int, height: int, width: int, planes: int, seed: int,
                  device="cpu", generator_device="cpu") -> torch.Tensor:
    """Stereo-Magnification-style synthetic MPI [B,H,W,P,4]: rgb U[-1,1) (tanh domain),
    alpha U[0,1), plane-0 alpha == 1."""
    g = torch.Generator(device=generator_device).manual_seed(seed)
    mpi = torch.rand((batch, height, width, planes, 4), generator=g,
                     dtype=torch.float32, device=generator_device)
    mpi[..., :3].mul_(2.0).sub_(1.0)
    mpi[:, :, :, 0, 3] = 1.0
    return mpi.to(device)


# ---------------------------------------------------------------------------
# BASELINE.json configs
# ---------------------------------------------------------------------------

def config1_camera():
    """C1: repo test MPI (test/rgba_00..09.png, 640x400, 10 planes)."""
    W, H = 640, 400
    f = focal_from_fov(W)
    K = intrinsics_matrix(f, f, W / 2.0, H / 2.0)
    poses = [pose_from(rot_y(1.0), (0.05, -0.02, 0.03)),
             pose_from(rot_y(-2.5), (-0.08, 0.03, -0.05))]
    return dict(H=H, W=W, P=10, K=K, poses=poses, depths=inv_depths(1, 100, 10))


def config2():
    """C2: 32-plane 1024x576 MPI, batch of 64 target views (MPI broadcast)."""
    W, H, P = 1024, 576, 32
    f = focal_from_fov(W)
    return dict(H=H, W=W, P=P, K=intrinsics_matrix(f, f, W / 2.0, H / 2.0),
                poses=sway_path(64), depths=inv_depths(1, 100, P), seed=0)


def config3():
    """C3: plane-sweep volume, 5 source 1024x768 images -> 64 depth planes."""
    W, H, D, S = 1024, 768, 64, 5
    f = focal_from_fov(W)
    poses = [pose_from(rot_y(0.5 * (i - 2)), (0.05 * (i - 2), 0.01, 0.0)) for i in range(S)]
    return dict(H=H, W=W, D=D, S=S, K=intrinsics_matrix(f, f, W / 2.0, H / 2.0),
                poses=poses, depths=inv_depths(1, 100, D), seed=1)


def config4(n_poses: int = 1000):
    """C4: 128-plane 1024x1024 MPI, 1000-pose camera path (view-sharded)."""
    W = H = 1024
    P = 128
    f = focal_from_fov(W)
    return dict(H=H, W=W, P=P, K=intrinsics_matrix(f, f, W / 2.0, H / 2.0),
                poses=sway_path(n_poses), depths=inv_depths(1, 100, P), seed=0)


def config5():
    """C5: 256-plane 4096x2160 MPI, plane-sharded, one pose."""
    W, H, P = 4096, 2160, 256
    f = focal_from_fov(W)
    return dict(H=H, W=W, P=P, K=intrinsics_matrix(f, f, W / 2.0, H / 2.0),
                poses=[pose_from(rot_y(1.0), (0.05, -0.02, 0.03))],
                depths=inv_depths(1, 100, P), seed=0)


# Phase tags of bench.py's timed regions (mpiv_mark: an empty marker kernel of tag x 64 work-items
# launched before each region; tools/parse_prof.py files every later dispatch under the last
# marker's tag, so the rocprof summary separates legs that launch the same kernel and grid).
PROF_TAGS = {"untimed": 1, "c4": 2, "sv": 3, "c2": 4, "c3_dropin": 5, "c3": 6, "c3_ten": 7, "nb": 8,
             "netout": 9, "u8_sv": 10, "u8_mv": 11, "u8_kernel": 12, "train_fwd": 13, "train_inf": 14,
             "train_inf_dropin": 15, "train_bwd": 16, "train_bwd_nockpt": 17, "train_bwd_minws": 18, "c5": 19,
             "c5_kernel": 20, "nt_fused": 21, "nt_two_step": 22}

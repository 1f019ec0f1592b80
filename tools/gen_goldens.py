#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
`utils.py` (Findeton/mpi-vision, /root/reference) on CPU in this container.

This is test tooling only: it runs where /root/reference exists and is never
imported by the package, the tests, bench.py or smoke().  The committed
outputs are data (inputs + expected outputs + exact fp32 matrices).

How the reference is imported: fastbook / fastai /
torchvision are not installed, so tools/refstub/ provides import stubs that
only re-export names (os, np, torch, Tensor, Module, Path); utils.py is loaded
with importlib and its module-global `device` is rebound to CPU.  All the
hot-path arithmetic is torch 2.10.0 CPU (MKL), exactly as the reference runs
it.

Usage:  python tools/gen_goldens.py [--skip-large]
"""
from __future__ import annotations

import argparse
import hashlib
import importlib.util
import json
import math
import os
import sys
import time
import warnings

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from mpi_vision_amd import configs  # noqa: E402  (pure-python workload definitions)


def load_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REPO, "tools", "refstub"))
    spec = importlib.util.spec_from_file_location("ref_utils", os.path.join(REF, "utils.py"))
    mod = importlib.util.module_from_spec(spec)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec.loader.exec_module(mod)
    mod.device = torch.device("cpu")
    return mod


def sha(t: torch.Tensor) -> str:
    return hashlib.sha256(t.contiguous().numpy().tobytes()).hexdigest()


def samples(t: torch.Tensor, n: int = 8192, seed: int = 1234):
    flat = t.contiguous().reshape(-1)
    idx = np.random.default_rng(seed).integers(0, flat.numel(), size=min(n, flat.numel()))
    return idx.astype(np.int64), flat[torch.from_numpy(idx)].numpy().copy()


def f32(x):
    return configs.f32(x)


def homographies(ref, pose, depths, K):
    """The reference's H, built with the same shapes/op sequence it uses inside
    mpi_render_view_torch -> projective_forward_homography_torch -> planar_transform_torch
    (utils.py:278-285, 255-262, 218-229) and inv_homography_torch (utils.py:44-67)."""
    B = pose.shape[0]
    P = depths.shape[0]
    d = depths.reshape([P, 1]).repeat(1, B)
    rot = pose[:, :3, :3]
    t = pose[:, :3, 3:]
    n_hat = torch.Tensor([0., 0., 1.]).reshape([1, 1, 1, 3]).repeat([P, B, 1, 1])
    a = -torch.reshape(d, [P, B, 1, 1])
    rep = [P, 1, 1, 1]
    k = torch.unsqueeze(K, 0).repeat(rep)
    H = ref.inv_homography_torch(k, k, torch.unsqueeze(rot, 0).repeat(rep),
                                 torch.unsqueeze(t, 0).repeat(rep), n_hat, a)
    return H  # [P, B, 3, 3]


def rand_pose(g, rot_scale, t_scale):
    """Random rigid pose from an axis-angle draw (float64 math, rounded once)."""
    v = (torch.rand(3, generator=g, dtype=torch.float64) * 2 - 1) * rot_scale
    th = float(v.norm())
    kx, ky, kz = (v / th).tolist() if th > 0 else (0.0, 0.0, 1.0)
    c, s, C = math.cos(th), math.sin(th), 1 - math.cos(th)
    R = [[c + kx * kx * C, kx * ky * C - kz * s, kx * kz * C + ky * s],
         [ky * kx * C + kz * s, c + ky * ky * C, ky * kz * C - kx * s],
         [kz * kx * C - ky * s, kz * ky * C + kx * s, c + kz * kz * C]]
    t = ((torch.rand(3, generator=g, dtype=torch.float64) * 2 - 1) * t_scale).tolist()
    return configs.pose_from(R, t)


def small_cases(ref):
    out = {}
    meta = {}

    # inv_depths (utils.py:297-318), exact doubles
    for n in (1, 2, 3, 10, 32, 64, 128, 256):
        out[f"inv_depths_{n}"] = np.array(ref.inv_depths(1, 100, n), dtype=np.float64)
    out["inv_depths_0.5_20_7"] = np.array(ref.inv_depths(0.5, 20.0, 7), dtype=np.float64)

    g = torch.Generator().manual_seed(7)

    # inv_homography_torch / render homographies
    K2 = f32([configs.intrinsics_matrix(150.0, 171.5, 60.25, 40.5),
              configs.intrinsics_matrix(133.0, 120.0, 70.0, 33.0)])
    poses2 = f32([rand_pose(g, 0.3, 0.4), rand_pose(g, 0.2, 0.5)])
    dep5 = f32(ref.inv_depths(1, 100, 5))
    out["hom_K"], out["hom_pose"], out["hom_depths"] = K2.numpy(), poses2.numpy(), dep5.numpy()
    out["hom_H"] = homographies(ref, poses2, dep5, K2).numpy()

    # --- render cases -------------------------------------------------------
    def render_case(name, B, H, W, P, seed, K, poses, depths, broadcast=False, alpha_fn=None):
        mpi = configs.synthetic_mpi(1 if broadcast else B, H, W, P, seed)
        if alpha_fn is not None:
            alpha_fn(mpi)
        mpi_in = mpi.expand(B, H, W, P, 4) if broadcast else mpi
        res = ref.mpi_render_view_torch(mpi_in, poses, depths, K)
        out[f"{name}_K"], out[f"{name}_pose"], out[f"{name}_depths"] = K.numpy(), poses.numpy(), depths.numpy()
        out[f"{name}_H"] = homographies(ref, poses, depths, K).numpy()
        out[f"{name}_out"] = res.numpy()
        meta[name] = dict(B=B, H=H, W=W, P=P, seed=seed, broadcast=broadcast,
                          mpi_sha=sha(mpi), alpha_fn=None if alpha_fn is None else alpha_fn.__name__)

    # mild motion, fx != fy, off-centre principal point, B=2 (independent MPIs)
    Kr = f32([configs.intrinsics_matrix(120.0, 131.0, 60.0, 37.5),
              configs.intrinsics_matrix(118.5, 118.5, 66.0, 33.0)])
    pr = f32([configs.pose_from(configs.rot_y(3.0), (0.1, -0.05, 0.08)),
              rand_pose(g, 0.05, 0.1)])
    render_case("render_a", 2, 72, 128, 8, 11, Kr, pr, f32(ref.inv_depths(1, 100, 8)))
    # large motion: planes partly behind the camera / far out of bounds
    pl = f32([rand_pose(g, 0.9, 1.5), rand_pose(g, 0.6, 3.0)])
    render_case("render_big", 2, 72, 128, 8, 12, Kr, pl, f32(ref.inv_depths(0.5, 10, 8)))
    # odd sizes, broadcast MPI over a batch of 3 poses
    Ko = f32([configs.intrinsics_matrix(44.0, 47.0, 26.0, 18.0)] * 3)
    po = f32([rand_pose(g, 0.1, 0.2) for _ in range(3)])
    render_case("render_odd", 3, 37, 53, 5, 13, Ko, po, f32(ref.inv_depths(1, 100, 5)),
                broadcast=True)

    def binary_alpha(m):
        m[..., 3] = (m[..., 3] > 0.5).float()
        m[:, :, :, 0, 3] = 1.0

    # alpha exactly 0 / 1 (transmittance edge cases), single plane-0-only check
    render_case("render_bin", 1, 40, 40, 4, 14, f32([configs.intrinsics_matrix(40.0, 40.0, 20.0, 20.0)]),
                f32([rand_pose(g, 0.05, 0.1)]), f32([9.0, 4.0, 2.0, 1.0]), alpha_fn=binary_alpha)
    render_case("render_p1", 1, 24, 33, 1, 15, f32([configs.intrinsics_matrix(30.0, 30.0, 16.0, 12.0)]),
                f32([rand_pose(g, 0.05, 0.1)]), f32([3.0]))

    # --- plane sweep ------------------------------------------------------------
    def psv_inputs(B, H, W, C, seed):
        gg = torch.Generator().manual_seed(seed)
        return torch.rand((B, H, W, C), generator=gg, dtype=torch.float32)

    img = psv_inputs(2, 48, 64, 3, 21)
    Kp = f32([configs.intrinsics_matrix(60.0, 63.0, 32.0, 24.0),
              configs.intrinsics_matrix(58.0, 58.0, 30.0, 26.0)])
    pp = f32([rand_pose(g, 0.08, 0.3), rand_pose(g, 0.05, 0.2)])
    dp = ref.inv_depths(1, 100, 6)
    res = ref.plane_sweep_torch(img, dp, pp, Kp)
    out.update(psv_a_K=Kp.numpy(), psv_a_pose=pp.numpy(), psv_a_depths=np.array(dp), psv_a_out=res.numpy())
    meta["psv_a"] = dict(B=2, H=48, W=64, C=3, seed=21, img_sha=sha(img))

    img1 = psv_inputs(1, 40, 40, 4, 22)[0]
    K1 = f32(configs.intrinsics_matrix(45.0, 45.0, 20.0, 20.0))
    p1 = f32(rand_pose(g, 0.05, 0.2))
    d1 = ref.inv_depths(0.8, 30, 5)
    res = ref.plane_sweep_torch_one(img1, d1, p1, K1)
    out.update(psv_one_K=K1.numpy(), psv_one_pose=p1.numpy(), psv_one_depths=np.array(d1), psv_one_out=res.numpy())
    meta["psv_one"] = dict(H=40, W=40, C=4, seed=22, img_sha=sha(img1))

    img2 = psv_inputs(1, 48, 64, 3, 23)[0]
    Ks = f32(configs.intrinsics_matrix(70.0, 72.0, 32.0, 24.0))
    Kt = f32(configs.intrinsics_matrix(80.0, 80.0, 80.0, 18.0))
    p2 = f32(rand_pose(g, 0.06, 0.25))
    d2 = ref.inv_depths(1, 50, 4)
    res = ref.plane_sweep_torch_one2(img2, d2, p2, Ks, Kt, 36, 160)
    out.update(psv_two_Ks=Ks.numpy(), psv_two_Kt=Kt.numpy(), psv_two_pose=p2.numpy(),
               psv_two_depths=np.array(d2), psv_two_out=res.numpy())
    meta["psv_two"] = dict(H=48, W=64, C=3, seed=23, tgt_h=36, tgt_w=160, img_sha=sha(img2))

    # --- format_network_input_torch (multi-source PSV + ref image), utils.py:473-498
    gf = torch.Generator().manual_seed(41)
    ref_img = torch.rand((2, 24, 32, 3), generator=gf)
    src_imgs = torch.rand((2, 24, 32, 6), generator=gf)   # two PSV sources
    ref_pose = f32([rand_pose(g, 0.05, 0.2), rand_pose(g, 0.05, 0.2)])
    src_poses = f32([[rand_pose(g, 0.05, 0.2), rand_pose(g, 0.05, 0.2)] for _ in range(2)])  # [B,2,4,4]
    Kf = f32([configs.intrinsics_matrix(30.0, 31.0, 16.0, 12.0), configs.intrinsics_matrix(29.0, 29.0, 15.5, 12.5)])
    planes_f = ref.inv_depths(1, 50, 4)
    res = ref.format_network_input_torch(None, ref_img, src_imgs, ref_pose, src_poses, planes_f, Kf)
    out.update(fni_ref=ref_img.numpy(), fni_src=src_imgs.numpy(), fni_ref_pose=ref_pose.numpy(),
               fni_src_poses=src_poses.numpy(), fni_K=Kf.numpy(), fni_planes=np.array(planes_f), fni_out=res.numpy())

    # --- camera-path I/O (utils.py:535-598, 689-721): RealEstate10K-style camera file
    lines = ["https://www.youtube.com/watch?v=abcDEF123_x"]
    gc = np.random.default_rng(5)
    for k in range(4):
        vals = [str(1000000 + 33366 * k)] + [repr(float(v)) for v in gc.uniform(0.3, 0.9, 4)] + ["0.0", "0.0"] + \
               [repr(float(v)) for v in gc.uniform(-1, 1, 12)]
        lines.append(" ".join(vals))
    cam_txt = "\n".join(["# a comment line"] + lines) + "\n"
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as fh:
        fh.write(cam_txt)
    read_back = ref.read_file_lines(fh.name)
    os.unlink(fh.name)
    parsed = ref.parse_camera_lines(read_back)
    meta["camera"] = dict(text=cam_txt, read_file_lines=read_back, parsed=parsed)
    intr = torch.Tensor([[0.5, 0.0, 0.5], [0.0, 0.6, 0.45], [0.0, 0.0, 1.0]])
    out.update(cam_scaled=ref.scale_intrinsics(intr, 400, 640).numpy(),
               cam_make=ref.make_intrinsics_matrix(554.25, 560.5, 320.0, 200.0).numpy())
    gq = torch.Generator().manual_seed(51)
    out.update(pre_in=torch.rand((2, 5, 6, 3), generator=gq).numpy())
    out.update(pre_out=ref.preprocess_image_torch(torch.tensor(out["pre_in"])).numpy())
    dep_in = torch.rand((2, 5, 6, 3), generator=gq) * 2.2 - 1.1
    out.update(dep_in=dep_in.numpy(), dep_out=ref.deprocess_image_torch(dep_in).numpy())

    # --- sampler wrappers -------------------------------------------------------
    gs = torch.Generator().manual_seed(31)
    imgs = torch.rand((2, 3, 20, 25, 4), generator=gs)
    coords = torch.rand((2, 3, 15, 10, 2), generator=gs) * 1.6 - 0.3
    coords[0, 0, 0, 0] = torch.tensor([0.0, 0.0])
    coords[0, 0, 0, 1] = torch.tensor([1.0, 1.0])
    coords[0, 0, 0, 2] = torch.tensor([-5.0, 0.5])
    coords[0, 0, 0, 3] = torch.tensor([0.5, 7.0])
    res = ref.bilinear_wrapper_torch(imgs, coords)
    out.update(bil_imgs=imgs.numpy(), bil_coords=coords.numpy(), bil_out=res.numpy())
    rimgs = torch.rand((2, 20, 25, 3), generator=gs)
    rcoords = torch.rand((2, 15, 10, 2), generator=gs) * 1.6 - 0.3
    res = ref.resampler_wrapper_torch(rimgs, rcoords)
    out.update(res_imgs=rimgs.numpy(), res_coords=rcoords.numpy(), res_out=res.numpy())

    # --- over_composite -----------------------------------------------------------
    layers = [torch.rand((2, 16, 24, 4), generator=gs) for _ in range(5)]
    res = ref.over_composite(layers)
    out.update(over_in=torch.stack(layers).numpy(), over_out=res.numpy())

    # --- per-pixel geometry helpers -------------------------------------------------
    pts = torch.rand((2, 3, 9, 11, 3), generator=gs) * 100 - 20
    pts[..., 2] = torch.rand((2, 3, 9, 11), generator=gs) * 2 - 0.5
    pts[0, 0, 0, 0, 2] = 0.0
    hh = torch.rand((2, 3, 3, 3), generator=gs) * 2 - 1
    tp = ref.transform_points_torch(pts, hh)
    out.update(tp_pts=pts.numpy(), tp_H=hh.numpy(), tp_out=tp.numpy())
    nh_in = tp.clone()
    nh_in[0, 0, 0, 0, 2] = 0.0
    nh_ref_in = nh_in.clone()
    nh = ref.normalize_homogeneous_torch(nh_ref_in)
    out.update(nh_in=nh_in.numpy(), nh_out=nh.numpy(), nh_in_after=nh_ref_in.numpy())

    depth = torch.rand((2, 6, 7), generator=gs) * 10 + 0.5
    pix = ref.meshgrid_abs_torch(2, 6, 7)
    Kc = f32([configs.intrinsics_matrix(20.0, 21.0, 3.0, 3.5), configs.intrinsics_matrix(19.0, 19.0, 3.2, 2.9)])
    cam = ref.pixel2cam_torch(depth, pix, Kc)
    proj = torch.rand((2, 4, 4), generator=gs)
    c2p = ref.cam2pixel_torch(cam, proj)
    out.update(p2c_depth=depth.numpy(), p2c_K=Kc.numpy(), p2c_out=cam.numpy(),
               c2p_proj=proj.numpy(), c2p_out=c2p.numpy())
    return out, meta


def large_cases(ref, meta_out):
    res = {}

    # C1: repo test MPI, two poses, full 400x640
    from PIL import Image
    planes = []
    for i in range(10):
        im = np.array(Image.open(os.path.join(OUT, "test_mpi", f"rgba_{i:02d}.png")))
        planes.append(torch.tensor(im).float() / 255)
    mpi = torch.stack(planes, dim=2).unsqueeze(0)  # [1, 400, 640, 10, 4]
    c1 = configs.config1_camera()
    K = f32([c1["K"]] * 2)
    poses = f32(c1["poses"])
    depths = f32(ref.inv_depths(1, 100, 10))
    mpi2 = mpi.expand(2, *mpi.shape[1:])
    t0 = time.time()
    out = ref.mpi_render_view_torch(mpi2, poses, depths, K)
    print(f"c1 render {time.time() - t0:.2f}s")
    idx, val = samples(out)
    res["c1_out"] = out.numpy()
    res["c1_H"] = homographies(ref, poses, depths, K).numpy()
    res.update(c1_K=K.numpy(), c1_pose=poses.numpy(), c1_depths=depths.numpy(),
               c1_idx=idx, c1_val=val)
    meta_out["c1"] = dict(mpi_sha=sha(mpi), out_sha=sha(out), shape=list(out.shape))

    # C2: 32-plane 1024x576, three of the 64 sway poses in one broadcast batch
    c2 = configs.config2()
    sel = [0, 21, 42]
    mpi = configs.synthetic_mpi(1, c2["H"], c2["W"], c2["P"], c2["seed"])
    poses = f32([c2["poses"][i] for i in sel])
    K = f32([c2["K"]] * len(sel))
    depths = f32(ref.inv_depths(1, 100, c2["P"]))
    t0 = time.time()
    out = ref.mpi_render_view_torch(mpi.expand(len(sel), *mpi.shape[1:]), poses, depths, K)
    print(f"c2 render {time.time() - t0:.2f}s")
    idx, val = samples(out)
    res.update(c2_H=homographies(ref, poses, depths, K).numpy(), c2_K=K.numpy(), c2_pose=poses.numpy(),
               c2_depths=depths.numpy(), c2_idx=idx, c2_val=val, c2_sel=np.array(sel))
    meta_out["c2"] = dict(mpi_sha=sha(mpi), out_sha=sha(out), shape=list(out.shape), sel=sel)
    del mpi, out

    # C3: PSV 5 x 768x1024x3 -> 64 planes
    c3 = configs.config3()
    gg = torch.Generator().manual_seed(c3["seed"])
    img = torch.rand((c3["S"], c3["H"], c3["W"], 3), generator=gg, dtype=torch.float32)
    poses = f32(c3["poses"])
    K = f32([c3["K"]] * c3["S"])
    t0 = time.time()
    out = ref.plane_sweep_torch(img, c3["depths"], poses, K)
    print(f"c3 psv {time.time() - t0:.2f}s")
    idx, val = samples(out)
    res.update(c3_K=K.numpy(), c3_pose=poses.numpy(), c3_depths=np.array(c3["depths"]), c3_idx=idx, c3_val=val)
    meta_out["c3"] = dict(img_sha=sha(img), out_sha=sha(out), shape=list(out.shape),
                          per_source_sha=[sha(out[i]) for i in range(out.shape[0])])
    del img, out

    # C4: 128-plane 1024^2, poses 0 and 500 of the 1000-pose path
    c4 = configs.config4()
    mpi = configs.synthetic_mpi(1, c4["H"], c4["W"], c4["P"], c4["seed"])
    depths = f32(ref.inv_depths(1, 100, c4["P"]))
    meta_out["c4"] = dict(mpi_sha=sha(mpi), sel=[0, 500], out_sha=[])
    for j, pi in enumerate((0, 500)):
        poses = f32([c4["poses"][pi]])
        K = f32([c4["K"]])
        t0 = time.time()
        out = ref.mpi_render_view_torch(mpi, poses, depths, K)
        print(f"c4 render pose {pi} {time.time() - t0:.2f}s")
        idx, val = samples(out, seed=1234 + j)
        res.update({f"c4_{pi}_H": homographies(ref, poses, depths, K).numpy(), f"c4_{pi}_pose": poses.numpy(),
                    f"c4_{pi}_idx": idx, f"c4_{pi}_val": val})
        meta_out["c4"]["out_sha"].append(sha(out))
        del out
    res.update(c4_K=f32([c4["K"]]).numpy(), c4_depths=depths.numpy())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-large", action="store_true")
    args = ap.parse_args()
    torch.set_num_threads(8)
    ref = load_reference()
    small, meta = small_cases(ref)
    np.savez_compressed(os.path.join(OUT, "small.npz"), **small)
    meta_all = {"small": meta, "torch": torch.__version__,
                "note": "generated by tools/gen_goldens.py from /root/reference/utils.py on CPU"}
    if not args.skip_large:
        large_meta = {}
        large = large_cases(ref, large_meta)
        np.savez_compressed(os.path.join(OUT, "large.npz"), **large)
        meta_all["large"] = large_meta
    else:
        old = os.path.join(OUT, "meta.json")
        if os.path.exists(old):
            meta_all["large"] = json.load(open(old)).get("large", {})
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta_all, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden fixtures for the MPI assembly: the notebook's own
`mpi_from_net_output` (fast-torch-stereo-vision.ipynb cell 10 L79-111), run here on
CPU with torch 2.10 autograd.  The function lives in a notebook cell, not in utils.py,
so it is taken from the notebook JSON at generation time (ast: the def node of that
cell) and executed with `device = cpu`; nothing of it is copied into this repository.
Test tooling only; writes tests/golden/netout.npz:

    <case>_pred [B,2P+3,H,W], <case>_ref [B,H,W,3], <case>_P, <case>_rgba [B,H,W,P,4],
    <case>_drgba (random upstream gradient), <case>_dpred (autograd d rgba . drgba / d pred),
    <case>_dref (the same w.r.t. the reference image, run with ref_img requiring grad)

Also tests/golden/netout_train.npz: the reference's TRAINING path through the same two
functions -- the notebook's mpi_from_net_output composed with /root/reference/utils.py's
mpi_render_view_torch (the two lines of both losses, ipynb cell 12 L7-11 / L38-42), run
under torch 2.10 CPU autograd with the network output AND the reference image requiring
grad:

    <case>_pred, _ref, _pose, _K, _depths, _H (the reference's homographies, [P,B,3,3]),
    _out (frames), _dout (random upstream gradient), _dpred, _dref

Plane counts 8, 12, 17 and 32 cover one, two (partial) and several 8-plane checkpoint
chunks of the fused training forward.

Usage:  python tools/gen_goldens_netout.py
"""
from __future__ import annotations

import ast
import glob
import json
import os

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "netout.npz")


def load_notebook_function(name="mpi_from_net_output"):
    nb = json.load(open(glob.glob(os.path.join(REF, "*.ipynb"))[0]))
    for cell in nb["cells"]:
        src = "".join(cell["source"])
        if f"def {name}(" not in src:
            continue
        tree = ast.parse(src)
        for node in tree.body:
            if isinstance(node, ast.FunctionDef) and node.name == name:
                ns = {"torch": torch, "device": torch.device("cpu")}
                exec(compile(ast.Module(body=[node], type_ignores=[]), f"<notebook:{name}>", "exec"), ns)
                return ns[name]
    raise RuntimeError(f"{name} not found in the notebook")


def train_cases(fn):
    """The fused net-output render's training goldens (netout_train.npz, module docstring)."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from gen_goldens import f32, homographies, load_reference, rand_pose
    from mpi_vision_amd import configs
    ref = load_reference()
    g = torch.Generator().manual_seed(606)
    out = {}

    def case(name, B, H, W, P, rot, trans, f=None, scale=1.0):
        f = f or 0.9 * W
        pred = ((torch.rand((B, 2 * P + 3, H, W), generator=g) * 2 - 1) * scale).requires_grad_(True)
        img = (torch.rand((B, H, W, 3), generator=g) * 2 - 1).requires_grad_(True)
        K = f32([configs.intrinsics_matrix(f, f * 1.02, W / 2.0 - 0.5, H / 2.0 + 0.5)] * B)
        pose = f32([rand_pose(g, rot, trans) for _ in range(B)])
        depths = f32(ref.inv_depths(1, 100, P))
        rgba = fn(pred, {"mpi_planes": torch.zeros((B, P)), "ref_img": img})
        frames = ref.mpi_render_view_torch(rgba, pose, depths, K)
        dout = torch.rand(frames.shape, generator=g) * 2 - 1
        frames.backward(dout)
        out.update({f"{name}_pred": pred.detach().numpy(), f"{name}_ref": img.detach().numpy(),
                    f"{name}_pose": pose.numpy(), f"{name}_K": K.numpy(), f"{name}_depths": depths.numpy(),
                    f"{name}_H": homographies(ref, pose, depths, K).numpy(), f"{name}_out": frames.detach().numpy(),
                    f"{name}_dout": dout.numpy(), f"{name}_dpred": pred.grad.numpy(),
                    f"{name}_dref": img.grad.numpy()})

    case("ta", 2, 24, 40, 12, 0.03, 0.06)
    case("tb", 1, 33, 47, 17, 0.05, 0.1)           # odd sizes, three chunks (the last partial)
    case("tc", 1, 16, 24, 8, 0.02, 0.05)           # exactly one chunk
    case("td", 1, 20, 36, 32, 0.3, 0.5, scale=1.4)  # Stereo-Mag plane count, large motion, off-range values
    path = os.path.join(REPO, "tests", "golden", "netout_train.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items() if k.endswith("dpred")})


def main():
    fn = load_notebook_function()
    train_cases(fn)
    if os.environ.get("NETOUT_TRAIN_ONLY") == "1":
        return
    g = torch.Generator().manual_seed(2024)
    out = {}

    def case(name, B, H, W, P, scale=1.0):
        pred = ((torch.rand((B, 2 * P + 3, H, W), generator=g) * 2 - 1) * scale).requires_grad_(True)
        ref = torch.rand((B, H, W, 3), generator=g) * 2 - 1
        dep = {"mpi_planes": torch.zeros((B, P)), "ref_img": ref}
        rgba = fn(pred, dep)
        drgba = torch.rand(rgba.shape, generator=g) * 2 - 1
        rgba.backward(drgba)
        # the same with the reference image differentiable too: d ref (and d pred, unchanged)
        ref2 = ref.clone().requires_grad_(True)
        pred2 = pred.detach().clone().requires_grad_(True)
        fn(pred2, {"mpi_planes": dep["mpi_planes"], "ref_img": ref2}).backward(drgba)
        assert torch.equal(pred2.grad, pred.grad)
        out.update({f"{name}_pred": pred.detach().numpy(), f"{name}_ref": ref.numpy(),
                    f"{name}_P": np.array(P, np.int32), f"{name}_rgba": rgba.detach().numpy(),
                    f"{name}_drgba": drgba.numpy(), f"{name}_dpred": pred.grad.numpy(),
                    f"{name}_dref": ref2.grad.numpy()})

    case("na", 2, 24, 40, 6)
    case("nb", 1, 17, 29, 32)          # odd sizes, a Stereo-Mag plane count
    case("nc", 3, 8, 72, 3, scale=1.5)  # values outside the tanh range too
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items() if k.endswith("rgba")})


if __name__ == "__main__":
    main()

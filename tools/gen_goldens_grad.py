#!/usr/bin/env python3
"""Golden fixtures for the render BACKWARD: the reference's
autograd gradient of `mpi_render_view_torch` (utils.py:267-294) with respect to the
MPI, computed by running /root/reference/utils.py on CPU (torch 2.10.0 autograd:
over_composite's MulBackward/RsubBackward chain, utils.py:149-156, then
grid_sampler_2d_backward, utils.py:128).  Test tooling only (see gen_goldens.py for
how the reference is imported); writes tests/golden/grad.npz.

Also records the notebook's training-loss use (`test_loss`, ipynb cell 12 L5-15):
mpi_from_net_output (ipynb cell 10 L79-111, loaded from the notebook: it lives
there, not in utils.py) -> render -> MSE, differentiated w.r.t. the network output.

Usage:  python tools/gen_goldens_grad.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from gen_goldens import OUT, f32, homographies, load_reference, rand_pose  # noqa: E402
from mpi_vision_amd import configs  # noqa: E402


def mpi_from_net_output(mpi_pred, ref_img, num_mpi_planes):
    """The notebook's own mpi_from_net_output (ipynb cell 10 L79-111), taken from the
    notebook at generation time (gen_goldens_netout.load_notebook_function)."""
    from gen_goldens_netout import load_notebook_function
    fn = load_notebook_function()
    B = mpi_pred.shape[0]
    return fn(mpi_pred, {"mpi_planes": torch.zeros((B, num_mpi_planes)), "ref_img": ref_img})


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    out = {}
    g = torch.Generator().manual_seed(77)

    def case(name, B, H, W, P, seed, K, poses, depths, broadcast=False, alpha_fn=None):
        mpi = configs.synthetic_mpi(1 if broadcast else B, H, W, P, seed)
        if alpha_fn is not None:
            alpha_fn(mpi)
        leaf = mpi.clone().requires_grad_(True)
        inp = leaf.expand(B, H, W, P, 4) if broadcast else leaf
        res = ref.mpi_render_view_torch(inp, poses, depths, K)
        dout = torch.rand(res.shape, generator=g) * 2 - 1
        res.backward(dout)
        out.update({f"{name}_mpi": mpi.numpy(), f"{name}_pose": poses.numpy(), f"{name}_K": K.numpy(),
                    f"{name}_depths": depths.numpy(), f"{name}_H": homographies(ref, poses, depths, K).numpy(),
                    f"{name}_out": res.detach().numpy(), f"{name}_dout": dout.numpy(),
                    f"{name}_grad": leaf.grad.numpy()})

    Ka = f32([configs.intrinsics_matrix(60.0, 63.0, 28.0, 19.5), configs.intrinsics_matrix(58.0, 58.0, 30.0, 21.0)])
    pa = f32([configs.pose_from(configs.rot_y(2.0), (0.06, -0.03, 0.05)), rand_pose(g, 0.04, 0.08)])
    case("ga", 2, 40, 56, 6, 31, Ka, pa, f32(ref.inv_depths(1, 100, 6)))
    Kb = f32([configs.intrinsics_matrix(40.0, 42.0, 24.0, 18.0)])
    case("gbig", 1, 36, 48, 5, 32, Kb, f32([rand_pose(g, 0.8, 1.5)]), f32(ref.inv_depths(0.5, 10, 5)))

    def binary_alpha(m):
        m[..., 3] = (m[..., 3] > 0.5).float()
        m[:, :, :, 0, 3] = 1.0

    Kc = f32([configs.intrinsics_matrix(32.0, 32.0, 16.0, 16.0)])
    case("gbin", 1, 32, 32, 4, 33, Kc, f32([rand_pose(g, 0.05, 0.1)]), f32([9.0, 4.0, 2.0, 1.0]),
         alpha_fn=binary_alpha)
    Kd = f32([configs.intrinsics_matrix(30.0, 31.0, 17.0, 11.0)] * 3)
    case("gbc", 3, 23, 35, 4, 34, Kd, f32([rand_pose(g, 0.05, 0.1) for _ in range(3)]),
         f32(ref.inv_depths(1, 100, 4)), broadcast=True)

    # notebook training loss (test_loss, ipynb cell 12 L5-15): d MSE / d network output
    B, H, W, P = 2, 32, 40, 5
    pred = (torch.rand((B, 2 * P + 3, H, W), generator=g) * 2 - 1).requires_grad_(True)
    ref_img = torch.rand((B, H, W, 3), generator=g) * 2 - 1
    tgt = torch.rand((B, H, W, 3), generator=g) * 2 - 1
    Kl = f32([configs.intrinsics_matrix(36.0, 36.0, 20.0, 16.0)] * B)
    pl = f32([rand_pose(g, 0.04, 0.1) for _ in range(B)])
    planes = f32(ref.inv_depths(1, 100, P))
    rgba = mpi_from_net_output(pred, ref_img, P)
    img = ref.mpi_render_view_torch(rgba, pl, planes, Kl)
    loss = torch.nn.functional.mse_loss(img, tgt)
    loss.backward()
    out.update(loss_pred=pred.detach().numpy(), loss_ref=ref_img.numpy(), loss_tgt=tgt.numpy(),
               loss_K=Kl.numpy(), loss_pose=pl.numpy(), loss_planes=planes.numpy(),
               loss_value=np.array(loss.item(), np.float32), loss_grad=pred.grad.numpy(),
               loss_H=homographies(ref, pl, planes, Kl).numpy())
    np.savez_compressed(os.path.join(OUT, "grad.npz"), **out)
    print("wrote", os.path.join(OUT, "grad.npz"), {k: v.shape for k, v in out.items() if k.endswith("grad")})


if __name__ == "__main__":
    main()

"""Host cost of PyTorch's autograd machinery around the drop-in's training step at the notebook shape
(224x224, 10 planes): a custom autograd.Function that launches nothing (identity forward / backward on a
ROCm tensor) against the render's RenderFunction, each piece timed on the host (perf_counter, no sync).
Probe only (GPU box): python tools/probes/autograd_floor_probe.py > gpurun_out/autograd_probe.json"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mpi_vision_amd as mv  # noqa: E402
from mpi_vision_amd import _host, _lib, configs  # noqa: E402

dev = torch.device("cuda:0")
N, P, n = 224, 10, 300
f = configs.focal_from_fov(N)
K = configs.f32(configs.intrinsics_matrix(f, f, N / 2.0, N / 2.0)).to(dev)[None]
pose = configs.f32(configs.pose_from(configs.rot_y(1.0), (0.05, -0.02, 0.03))).to(dev)[None]
planes = configs.f32(mv.inv_depths(1, 100, P)).to(dev)
leaf = configs.synthetic_mpi(1, N, N, P, 9).to(dev).requires_grad_(True)
dout = torch.rand((1, N, N, 3), device=dev)
homs = _host.render_homographies_device(pose, planes, K, 1)


class Ident(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g


small = torch.zeros(4, device=dev, requires_grad=True)
gsmall = torch.ones(4, device=dev)


def host_us(fn, k=n):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        fn()
    h = (time.perf_counter() - t) / k * 1e6
    torch.cuda.synchronize()
    return h


def ident_step():
    Ident.apply(small).backward(gsmall)
    small.grad = None


def render_apply():
    return _lib.RenderFunction.apply(leaf, homs)


def render_step_fixed_homs():
    render_apply().backward(dout)
    leaf.grad = None


def dropin_step():
    mv.mpi_render_view_torch(leaf, pose, planes, K).backward(dout)
    leaf.grad = None


ck = _lib.render_train(leaf.detach(), homs)[1]
res = {"ident_fwd_bwd_host_us": host_us(ident_step),
       "render_apply_host_us": host_us(render_apply),
       "render_step_fixed_homs_host_us": host_us(render_step_fixed_homs),
       "dropin_step_host_us": host_us(dropin_step),
       "render_backward_direct_host_us": host_us(lambda: _lib.render_backward(leaf.detach(), homs, dout, ckpt=ck)),
       "render_backward_nomon_host_us": host_us(lambda: _lib.render_backward(leaf.detach(), homs, dout, ckpt=ck,
                                                                          check=False)),
       "torch_empty_us": host_us(lambda: torch.empty((1, N, N, P, 4), device=dev)),
       "homs_device_us": host_us(lambda: _host.render_homographies_device(pose, planes, K, 1))}
print(json.dumps({k: round(v, 2) for k, v in res.items()}))

# where the autograd backward's time goes: timestamps around render_backward inside the engine's call
marks = []
orig = _lib.render_backward


def traced(*a, **k):
    marks.append(("rb_in", time.perf_counter()))
    r = orig(*a, **k)
    marks.append(("rb_out", time.perf_counter()))
    return r


_lib.render_backward = traced
spans = {"apply": [], "to_rb": [], "rb": [], "after_rb": [], "grad_none": []}
for i in range(n + 10):
    marks.clear()
    t0 = time.perf_counter()
    o = render_apply()
    t1 = time.perf_counter()
    o.backward(dout)
    t2 = time.perf_counter()
    leaf.grad = None
    t3 = time.perf_counter()
    if i >= 10:
        d = dict(marks)
        spans["apply"].append(t1 - t0)
        spans["to_rb"].append(d["rb_in"] - t1)
        spans["rb"].append(d["rb_out"] - d["rb_in"])
        spans["after_rb"].append(t2 - d["rb_out"])
        spans["grad_none"].append(t3 - t2)
_lib.render_backward = orig
torch.cuda.synchronize()
import statistics  # noqa: E402
print(json.dumps({k: round(statistics.median(v) * 1e6, 2) for k, v in spans.items()}))

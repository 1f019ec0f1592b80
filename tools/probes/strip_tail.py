#!/usr/bin/env python3
"""Tail-effect probe for the in-place render (render_chunk_strip_kernel<16, 2>): the same per-pixel work
at frame heights whose block counts are / are not whole multiples of the blocks resident at once
(256 CUs x 3 = 768; a 32 x 16 tile per block; square frames, whose unit scale keeps the per-pixel work
the same).  Prints the time
per megapixel; a partial last round of blocks shows up as a higher per-pixel time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mpi_vision_amd import _host, _lib, configs  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    c = configs.config4()
    P = 96  # 1152^2 x 96 planes stays under the in-place kernel's 2-GiB view span
    depths = configs.f32(configs.inv_depths(1, 100, P))
    for rep in range(2):
        for H in (960, 1024, 1088, 1152):  # square frames: the swapped normalisation keeps unit scale
            W = H
            g = torch.Generator(device=dev).manual_seed(0)
            mpi = torch.rand((1, H, W, P, 4), generator=g, device=dev)
            K = configs.f32([configs.intrinsics_matrix(c["K"][0][0], c["K"][1][1], W / 2.0, H / 2.0)])
            homs = _host.render_homographies(configs.f32(c["poses"][100:101]), depths, K, 1).to(dev)
            out = torch.empty((1, H, W, 3), device=dev)
            fn = lambda: _lib._call("mpiv_render", mpi, _lib._strides(mpi), 1, H, W, P, homs, out,  # noqa: E731
                                    _lib._stream(dev))
            for _ in range(100):
                fn()
            s = torch.cuda.current_stream()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(20):
                fn()
            b.record(s)
            b.synchronize()
            ms = a.elapsed_time(b) / 20
            blocks = ((W + 31) // 32) * ((H + 15) // 16)
            print(json.dumps({"H": H, "rep": rep, "route": _lib.route("render", 1, H, W, P)[0], "blocks": blocks, "rounds_of_768": round(blocks / 768, 3),
                              "ms": round(ms, 4), "ms_per_Mpix": round(ms / (H * W / 1e6), 4)}), flush=True)
            del mpi, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

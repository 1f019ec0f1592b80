"""Camera-path and frame-codec helpers around the hot path.

Host-side parsing of RealEstate10K-style camera files feeds real pose sequences
to the view-sharded renderer; the [-1,1] <-> uint8 frame codec runs as HIP
kernels.  Citations are into the reference utils.py.
"""
from __future__ import annotations

import torch

from . import _lib


def read_file_lines(filename):
    """Lines of a text file without their newlines, skipping lines that start with
    '#' (utils.py:583-598)."""
    with open(filename) as fh:
        return [line.replace("\n", "") for line in fh.readlines() if line[0] != "#"]


def parse_camera_lines(lines):
    """Parse a camera file (utils.py:689-721).  Line 0 is the video URL; every other
    line is `timestamp fx fy px py k1 k2 r00 r01 r02 t0 r10 .. t2` (19 fields).
    Returns {'youtube_id', 'timestamps', 'intrinsics', 'poses'}; poses are 4x4
    world-to-camera row lists.  Non-zero distortion (k1, k2) is rejected."""
    url = lines[0]
    rows = []
    for line in lines[1:]:
        fields = line.split(" ")
        rows.append([int(fields[0])] + [float(f) for f in fields[1:]])
    assert all(r[5] == 0.0 and r[6] == 0.0 for r in rows), "non-zero k1/k2 distortion"
    marker = "/watch?v="
    start = url.find(marker) + len(marker)
    return {
        "youtube_id": url[start:],
        "timestamps": [r[0] for r in rows],
        "intrinsics": [r[1:5] for r in rows],
        "poses": [[r[7:11], r[11:15], r[15:19], [0.0, 0.0, 0.0, 1.0]] for r in rows],
    }


def make_intrinsics_matrix(fx, fy, cx, cy):
    """3x3 pixel intrinsics on the module device (utils.py:576-581)."""
    from . import utils
    return torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float32).to(utils.device)


def scale_intrinsics(intrinsics, height, width):
    """Scale normalised intrinsics to pixels (utils.py:535-546): fx, cx by width;
    fy, cy by height."""
    scale = torch.tensor([[width, 1.0, width], [0.0, height, height], [0.0, 0.0, 1.0]], dtype=torch.float32)
    return intrinsics * scale.to(intrinsics.device)


def preprocess_image_torch(image):
    """[0,1] -> [-1,1]: image*2 - 1 (utils.py:334-342), HIP kernel."""
    return _lib.preprocess(image)


def deprocess_image_torch(image):
    """[-1,1] -> uint8 by truncation, ((x+1)/2)*255 converted like torch's CPU
    float->uint8 cast (truncate to int32, keep the low byte; out of int32 range or
    NaN -> 0), returned as a CPU ByteTensor like the reference (utils.py:344-352)."""
    return _lib.deprocess_u8(image).cpu()

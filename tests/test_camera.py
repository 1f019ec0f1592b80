"""Camera-path I/O (host) against the reference's parses of a synthetic camera file,
and the frame codec kernels (GPU) against the reference's outputs."""
import numpy as np
import pytest
import torch

import mpi_vision_amd as mv  # noqa: E402


def test_read_and_parse_camera_file(meta, tmp_path):
    cam = meta["small"]["camera"]
    f = tmp_path / "cams.txt"
    f.write_text(cam["text"])
    lines = mv.read_file_lines(str(f))
    assert lines == cam["read_file_lines"]
    parsed = mv.parse_camera_lines(lines)
    assert parsed == cam["parsed"]


def test_parse_rejects_distortion():
    with pytest.raises(AssertionError):
        mv.parse_camera_lines(["url", "1 0.5 0.5 0.5 0.5 0.1 0.0 " + " ".join(["0.0"] * 12)])


def test_scale_intrinsics(small):
    intr = torch.tensor([[0.5, 0.0, 0.5], [0.0, 0.6, 0.45], [0.0, 0.0, 1.0]])
    assert np.array_equal(mv.scale_intrinsics(intr, 400, 640).numpy(), small["cam_scaled"])


def test_make_intrinsics(small):
    mv.utils.device = torch.device("cpu")
    try:
        K = mv.make_intrinsics_matrix(554.25, 560.5, 320.0, 200.0)
    finally:
        mv.utils.device = torch.device("cuda")
    assert np.array_equal(K.numpy(), small["cam_make"])


@pytest.mark.gpu
def test_preprocess_deprocess(small, dev):
    pre = mv.preprocess_image_torch(torch.tensor(small["pre_in"]).to(dev))
    assert np.array_equal(pre.cpu().numpy(), small["pre_out"])
    dep = mv.deprocess_image_torch(torch.tensor(small["dep_in"]).to(dev))
    assert dep.device.type == "cpu" and dep.dtype == torch.uint8
    assert np.array_equal(dep.numpy(), small["dep_out"])
    edge = torch.tensor([-1.5, -0.5, 0.7, 255.9, 256.5, 300.7, -200.0, 1000.0, float("nan"), 3e9])
    want = ((((edge + 1.0) / 2.0) * 255)).type(torch.ByteTensor)
    got = mv.deprocess_image_torch(edge.to(dev))
    assert got.tolist() == want.tolist()

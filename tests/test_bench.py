"""bench.py's host logic on CPU: leg selection, the N-rank launcher (it must start the
ranks itself when the driver runs `bench.py --gpus N` outside torchrun, and refuse a
WORLD_SIZE that disagrees with --gpus), the host-core report of the CPU baseline, and
the library's route dry run that ties every leg to its rocprof dispatches."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from mpi_vision_amd import _lib, configs  # noqa: E402


def _parse(monkeypatch, *argv):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


def test_leg_selection(monkeypatch):
    assert _parse(monkeypatch).legs == list(bench.ALL_LEGS)
    assert _parse(monkeypatch, "--no-extras").legs == ["c4"]
    a = _parse(monkeypatch, "--no-config5", "--no-training", "--cpu-seconds", "0")
    assert a.legs == ["c4", "sv", "c2", "c3", "nb", "u8", "netout"]
    assert _parse(monkeypatch, "--legs", "c3").legs == ["c3"]
    with pytest.raises(SystemExit):
        _parse(monkeypatch, "--legs", "c9")


def test_spawn_ranks_runs_torchrun_child(monkeypatch):
    seen = {}

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 3)

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    assert bench.spawn_ranks(4) == 3
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")


def test_main_spawns_before_touching_the_gpu(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(bench, "spawn_ranks", lambda n: 7)
    monkeypatch.setattr(bench, "dist_setup", lambda a: (_ for _ in ()).throw(AssertionError("touched the GPU")))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.dist_setup(bench.parse())


def test_host_cores_report():
    threads, d = bench.host_cores()
    assert threads >= 1 and d["threads_used"] == threads
    assert d["host_nproc"] == os.cpu_count()
    assert threads <= d["affinity_cpus"]


def test_route_dry_run_names_the_launched_kernels():
    """mpiv_route reports the production kernel and grid without a GPU (no launch)."""
    assert _lib.route("render_packed", 1024, 1024, 128, 125) == ("render_rows_kernel<false, 6, true, false, 3, false, false>",
                                                                 16 * 43 * 125 * 256)
    assert _lib.route("render_packed", 1024, 1024, 128, 1)[0] == "render_rows_kernel<false, 4, true, false, 4, false, false>"
    # stretched frames (the swapped normalisation advances <= 0.8 texel rows per output row): same-row
    # tap reuse, R = 6, at every view count; one- and two-view launches also skip the south loads of rows
    # where every lane stayed (OOB)
    assert _lib.route("render_packed", 576, 1024, 32, 64)[0] == "render_rows_kernel<false, 6, true, false, 3, true, false>"
    assert _lib.route("render_packed", 576, 1024, 32, 8)[0] == "render_rows_kernel<false, 6, true, false, 3, true, false>"
    assert _lib.route("render_packed_ct", 2160, 4096, 32, 1)[0] == "render_rows_kernel<true, 6, true, false, 3, true, true>"
    assert _lib.route("render_packed_ct_rows", 2160, 4096, 32, 1, 0, 270)[0] == \
        "render_rows_kernel<true, 6, true, false, 3, true, true>"
    assert _lib.route("render_packed_ct_rows", 1024, 1024, 32, 125, 0, 128)[0] == \
        "render_rows_kernel<true, 6, true, false, 3, false, false>"
    # a stretched MPI in a small launch keeps the one-row kernel
    assert _lib.route("render_packed", 576, 1024, 32, 1)[0] == "render_packed_kernel<false, true>"
    assert _lib.route("plane_sweep", 5, 768, 1024, 3, 64, 768, 1024) == ("plane_sweep_dlane_kernel<3, true, 4, 3072, 2, false>",
                                                                         16 * 192 * 5 * 512)
    assert _lib.route("render", 1, 1024, 1024, 128) == ("render_chunk_strip_kernel<16, 2>", 32 * 64 * 256)
    assert _lib.route("render_train", 1, 1024, 1024, 128)[0] == "render_chunk_strip_kernel<16, 2>"
    with pytest.raises(RuntimeError, match="unknown entry"):
        _lib.route("nope", 1)
    with _lib.debug(render_tile=-1):
        with pytest.raises(RuntimeError, match="debug options"):
            _lib.route("render_packed", 64, 64, 4, 1)


def test_route_dry_run_u8_and_net_output():
    """The u8 texel render and the fused net-output render report their kernels (bench legs
    u8 / netout find their rocprof dispatches by them)."""
    # one view leaves the SIMDs 4 waves each: 4 rows in flight; the 125-view launch: 2
    assert _lib.route("render_packed_u8", 1024, 1024, 128, 1) == ("render_u8_kernel<false, 4, true, 4>",
                                                                  16 * 64 * 256)
    assert _lib.route("render_packed_u8", 1024, 1024, 128, 125)[0] == "render_u8_kernel<false, 4, true, 2>"
    name, grid = _lib.route("render_net_output", 1, 576, 1024, 32)
    assert name == "render_netout_kernel<8, 2, 1, true, true, true>" and grid == 576 * 512


def test_line_guard_prints_once():
    import io
    buf = io.StringIO()
    g = bench.LineGuard(0, out=buf)
    assert g.emit({"value": 1.0}) and not g.emit({"value": 2.0})
    assert buf.getvalue().count("\n") == 1 and '"value": 1.0' in buf.getvalue()
    other = io.StringIO()
    assert not bench.LineGuard(1, out=other).emit({"value": 1.0}) and other.getvalue() == ""


_HANG_WORKER = r"""
import os, sys, time
sys.path.insert(0, {repo!r})
import datetime
import torch.distributed as dist
import bench
rank = int(os.environ["RANK"])
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
res = {{"value": 123.0, "config5_plane_sharded": None}} if rank == 0 else {{}}
g = bench.LineGuard(rank)
g.arm(4.0, res, "config5_plane_sharded")
if bench.fault_injected("c5_hang", rank):
    time.sleep(1000)          # the last rank stops answering
dist.barrier()                # rank 0 blocks here: the exchange that never completes
res["config5_plane_sharded"] = {{"value": 1.0}}
g.emit(res)
"""


@pytest.mark.parametrize("world", [2, 3])
def test_line_guard_survives_a_hung_exchange(world, tmp_path):
    """A rank that stops answering in the collective leg (MPIV_BENCH_FAULT=c5_hang) must not cost the
    line: at the deadline rank 0 prints the complete line with the leg's error field and every rank
    exits 0 (gloo, CPU; the GPU-box rehearsal runs the same through bench.py's config-5 leg)."""
    import json
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    script = tmp_path / "w.py"
    script.write_text(_HANG_WORKER.format(repo=REPO))
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   MPIV_BENCH_FAULT="c5_hang")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert [p.returncode for p in procs] == [0] * world, [o[1][-500:] for o in outs]
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["value"] == 123.0 and "timed out" in line["config5_plane_sharded"]["error"]
    assert all(not any(ln.startswith("{") for ln in o[0].splitlines()) for o in outs[1:])


def test_sampled_boxes_cover_every_tap():
    """bench.sampled_boxes (the needed-bytes figure of configs 2 / 5): the map from output pixel to sample
    position is linear-fractional, so the frame corners bound it -- every tap of every pixel (computed
    here for all pixels) lies in the box, and the box is tight to one texel."""
    import numpy as np
    from mpi_vision_amd import _host, configs
    H, W, P, V = 23, 41, 6, 3
    g = __import__("torch").Generator().manual_seed(3)
    K = configs.f32([configs.intrinsics_matrix(40.0, 42.0, 20.0, 11.0)] * V)
    poses = configs.f32([configs.pose_from(configs.rot_y(3.0 * (i - 1)), (0.1 * i, -0.05, 0.02 * i)) for i in range(V)])
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 30, P)), K, V).numpy()
    box = bench.sampled_boxes(homs, H, W)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    h = homs.reshape(V, P, 3, 3).astype(np.float64)
    for v in range(V):
        for p in range(P):
            m = h[v, p]
            u = m[0, 0] * xs + m[0, 1] * ys + m[0, 2]
            vv = m[1, 0] * xs + m[1, 1] * ys + m[1, 2]
            w = m[2, 0] * xs + m[2, 1] * ys + m[2, 2]
            px = u / w * W / (H - 1) - 0.5
            py = vv / w * H / (W - 1) - 0.5
            x0, y0 = np.floor(px), np.floor(py)
            tx = np.concatenate([x0.ravel(), x0.ravel() + 1])
            ty = np.concatenate([y0.ravel(), y0.ravel() + 1])
            inside = (tx >= 0) & (tx < W) & (ty >= 0) & (ty < H)
            bx0, bx1, by0, by1 = box[v, p]
            if not inside.any():
                continue
            assert tx[inside].min() >= bx0 and tx[inside].max() <= bx1, (v, p)
            assert ty[inside].min() >= by0 and ty[inside].max() <= by1, (v, p)
            assert bx0 >= tx[inside].min() - 1 and bx1 <= tx[inside].max() + 1
    need = bench.needed_bytes(homs, H, W)
    assert need <= V * (P * H * W * 16 + H * W * 12)
    assert bench.needed_bytes(homs, H, W, union=True) <= need


def test_netout_needed_bytes_is_json_ready():
    """The net-output leg's needed-bytes figure is a plain int (the bench line is json.dumps'd) and sits
    between the frame alone and the formula's whole prediction."""
    import json
    from mpi_vision_amd import _host
    c = configs.config2()
    H, W, P = c["H"], c["W"], c["P"]
    homs = _host.render_homographies(configs.f32(c["poses"][5:6]), configs.f32(c["depths"]), configs.f32([c["K"]]), 1)
    need = bench.netout_needed_bytes(homs.numpy(), H, W)
    assert type(need) is int and json.dumps({"n": need})
    assert H * W * 12 < need < H * W * ((2 * P + 3) * 4 + 24)


def test_line_guard_serialises_numpy_scalars():
    import io
    import numpy as np
    buf = io.StringIO()
    g = bench.LineGuard(0, out=buf)
    assert g.emit({"value": np.float32(1.5), "n": np.int64(3)})
    assert '"value": 1.5' in buf.getvalue() and '"n": 3' in buf.getvalue()

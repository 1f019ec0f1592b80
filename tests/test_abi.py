"""CPU: the C-ABI library loads, exports every symbol include/mpiv.h declares, and
rejects bad arguments with error codes + messages (validated before any HIP call,
so this runs without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

from mpi_vision_amd import _lib  # noqa: E402

HEADER = os.path.join(REPO, "include", "mpiv.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(mpiv_\w+)\s*\(", text, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "mpiv_render" in syms and "mpiv_plane_sweep" in syms and len(syms) >= 15


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(declared_symbols()) <= set(_lib.EXPORTS)


def test_abi_version():
    assert _lib.load().mpiv_abi_version() == _lib.ABI_VERSION


@pytest.mark.parametrize("call", [
    ("mpiv_render", [None, None, 1, 4, 4, 2, None, None, None]),
    ("mpiv_render_packed", [None, 4, 4, 2, None, 1, None, None]),
    ("mpiv_plane_sweep", [None, None, 1, 4, 4, 3, None, None, None, 2, 4, 4, None, None]),
    ("mpiv_grid_sample", [None, None, 1, 1, 4, 4, None, None, 2, 2, None, None, None]),
    ("mpiv_over_composite", [None, 2, 4, 4, 1, None, None]),
    ("mpiv_combine_ct", [None, 2, 4, None, None]),
])
def test_null_pointers_rejected(call):
    name, args = call
    L = _lib.load()
    rc = getattr(L, name)(*args)
    assert rc == -1
    assert b"null pointer" in L.mpiv_last_error()


def test_bad_shapes_rejected():
    L = _lib.load()
    st = (ctypes.c_int64 * 5)(1, 1, 1, 1, 1)
    p = ctypes.c_void_p(16)
    assert L.mpiv_render(p, st, 0, 4, 4, 2, p, p, None) == -1
    assert b"bad shape" in L.mpiv_last_error()
    assert L.mpiv_render_packed_ct(p, 4, 4, 8, 5, 3, 0, p, 1, p, None) == -1
    assert b"plane range" in L.mpiv_last_error()
    assert L.mpiv_render_packed(ctypes.c_void_p(8), 4, 4, 2, p, 1, p, None) == -1
    assert b"alignment" in L.mpiv_last_error()


def test_build_id_matches_sources():
    """libmpiv.so carries the sha256 of the sources it was built from (csrc/SOURCES);
    _lib.load() refuses a library whose id differs from the tree's sources."""
    L = _lib.load()
    assert L.mpiv_build_id().decode() == _lib.source_hash()


def test_debug_options():
    """Kernel A/B variants are selected only through the debug entry point (no getenv on
    the launch path); unknown names are rejected; reset restores the defaults."""
    L = _lib.load()
    assert L.mpiv_debug_set(b"no_such_option", 1) == -1
    assert b"unknown option" in L.mpiv_last_error()
    with _lib.debug(render_mv=1, box_shrink=2):
        pass
    with pytest.raises(ValueError):
        with _lib.debug(bogus=1):
            pass


def test_ab_kernels_live_in_the_ab_library():
    """The production libmpiv.so carries only the routed kernels: options that pick a variant
    kept for A/B measurement are refused there, and _lib.debug() runs such blocks on
    libmpiv_ab.so (same sources, same build id, -DMPIV_AB=1), then returns to libmpiv.so."""
    L = _lib.load_main()
    for name, val in (("render_mv", 1), ("render_ring", 4), ("render_pair", 1), ("render_tile", 8),
                      ("render_vshare", 1), ("sweep_tile", 1), ("sweep_store", 2), ("render_chunk", 108),
                      ("sweep_dlane", 0), ("chunk_rows", 2), ("chunk_flight", 4), ("sweep_rows", 8),
                      ("bwd_gather", 1), ("bwd_gather", 2), ("chunk_strip", 2)):
        assert L.mpiv_debug_set(name.encode(), val) == -1, name
        assert b"libmpiv_ab.so" in L.mpiv_last_error()
    for name, val in (("render_tile", -1), ("render_vshare", 11), ("render_chunk", 4), ("chunk_rows", 1),
                      ("bwd_fallback", 1), ("box_shrink", 2), ("sweep_direct", 1), ("bwd_gather", 0),
                      ("chunk_strip", 0), ("chunk_strip", 1), ("u8_flight", 2), ("u8_flight", 4),
                      ("bwd_group", 8)):  # production kernels / test hooks
        assert L.mpiv_debug_set(name.encode(), val) == 0, name
    L.mpiv_debug_set(b"reset", 0)
    p = ctypes.c_void_p(256)
    assert L.mpiv_render_packed_lds(p, 8, 8, 2, p, 1, p, None) == -1
    assert b"libmpiv_ab.so" in L.mpiv_last_error()
    A = _lib.load_ab()
    assert A.mpiv_build_id().decode() == _lib.source_hash()
    with _lib.debug(render_mv=1):
        assert _lib.load() is A
    assert _lib.load() is L
    with _lib.debug(render_vshare=11):
        assert _lib.load() is L
    assert os.path.getsize(_lib.LIB_PATH) < os.path.getsize(_lib.AB_PATH)


@pytest.mark.parametrize("C", [1, 3, 4])
def test_plane_sweep_routes(C):
    """mpiv_route (dry run, no GPU): the sweep's production route by depth count -- the direct
    depth-per-lane kernel for D <= 2, the pixel-per-lane kernel (one block per 256 pixels of a
    row) for 3 <= D <= 8, the LDS-staged depth-per-lane kernel above (one pixel per lane and
    iteration up to D = 16); C > 4 the generic kernel."""
    B, Hs, Ws, Ht, Wt = 5, 768, 1024, 768, 1024
    for D in (1, 2, 3, 8, 9, 10, 64):
        name, grid = _lib.route("plane_sweep", B, Hs, Ws, C, D, Ht, Wt)
        if D <= 2:
            assert name == f"plane_sweep_direct_kernel<{C}>", (D, name)
        elif D <= 8:
            assert name == f"plane_sweep_px_kernel<{C}, 64>", (D, name)
            assert grid == (Wt // 256) * Ht * B * 256, (D, grid)
        else:  # one pixel per lane and iteration up to 16 depths, two above
            assert name == f"plane_sweep_dlane_kernel<{C}, true, 4, 3072, {1 if D <= 16 else 2}, false>", (D, name)
    assert _lib.route("plane_sweep", B, Hs, Ws, 5, 10, Ht, Wt)[0] == "plane_sweep_kernel"


def test_output_buffers_validated():
    """Caller-supplied outputs of the packed render / pack must be dense fp32 tensors of the
    exact shape on the same device, else a Python error (not out-of-bounds device writes)."""
    import torch
    good = torch.zeros(4)
    with pytest.raises(RuntimeError, match="out must be"):
        _lib._check_out(torch.zeros((2, 3)), (3, 2), good.device, "x")
    with pytest.raises(RuntimeError, match="out must be"):
        _lib._check_out(torch.zeros((3, 4))[:, :2], (3, 2), good.device, "x")
    with pytest.raises(RuntimeError, match="out must be"):
        _lib._check_out(torch.zeros((3, 2), dtype=torch.float64), (3, 2), good.device, "x")
    assert _lib._check_out(torch.zeros((3, 2)), (3, 2), good.device, "x") is not None


@pytest.mark.slow
def test_host_asan_builds():
    """Host AddressSanitizer + UBSan flavour (GPU ASan is not available on
    this pool): an ASan-instrumented libmpiv driven through every argument-validation
    path and the host homography chain, and the CPU oracle on small / degenerate inputs
    (tools/asan/Makefile, built into /tmp)."""
    import shutil
    import subprocess
    if shutil.which("/opt/rocm/bin/hipcc") is None or shutil.which("gcc") is None:
        pytest.skip("needs hipcc and gcc")
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tools", "asan"), "run"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "abi_check: 0 failure(s)" in r.stdout and "oracle_check: ok" in r.stdout


def test_backward_workspace_plane_groups():
    """mpiv_render_backward's smallest workspace holds one plane group's d samples (round 4):
    config 4 (1024x1024x128, 4 groups of 32 planes) fits in 1.5 GB, the one-group (fastest)
    size holds every plane's; a view under 2^25 plane-pixels is one group either way; the
    bwd_group test hook shrinks the groups (and the workspace) on demand."""
    L = _lib.load_main()
    full = L.mpiv_render_backward_workspace_size(1024, 1024, 128)
    small = L.mpiv_render_backward_workspace_size_min(1024, 1024, 128)
    assert 1.0e9 < small <= 1.5e9 < 1024 * 1024 * 128 * 16 < full, (small, full)
    one = L.mpiv_render_backward_workspace_size(64, 96, 12)
    assert one == L.mpiv_render_backward_workspace_size_min(64, 96, 12) > 64 * 96 * 12 * 16
    assert L.mpiv_debug_set(b"bwd_group", 8) == 0
    try:
        grouped = L.mpiv_render_backward_workspace_size(64, 96, 12)
    finally:
        L.mpiv_debug_set(b"reset", 0)
    assert grouped < one

"""CPU multi-process (gloo, world_size 2 and 3) tests of the sharding logic in
mpi_vision_amd/parallel.py.  Per-rank compute uses the oracle (test infrastructure);
what is under test is the product's exchange / ordering / gather logic, checked
against the single-device sequential render within 1e-5 (reassociation)."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(H=37, W=53, P=11):
    sys.path.insert(0, REPO)
    from mpi_vision_amd import _host, configs
    V = 2
    mpi = configs.synthetic_mpi(1, H, W, P, 5)
    K = configs.f32([configs.intrinsics_matrix(50.0, 52.0, 26.0, 18.0)] * V)
    poses = configs.f32([configs.pose_from(configs.rot_y(1.5), (0.05, -0.02, 0.03)),
                         configs.pose_from(configs.rot_y(-2.0), (-0.1, 0.02, 0.05))])
    depths = configs.f32(configs.inv_depths(1, 20, P))
    homs = _host.render_homographies(poses, depths, K, V).numpy()
    return mpi.expand(V, H, W, P, 4).numpy(), homs


def _plane_worker(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_vision_amd import parallel
    from oracle import oracle
    mpi, homs = _case()
    V, H, W, P, _ = mpi.shape
    p0, p1 = parallel.shard_range(P, rank, world)
    ct = torch.from_numpy(oracle.render_ct(mpi, homs, p0, p1, back=(rank == 0), nthreads=2))
    parts = parallel.exchange_bands(ct)
    band = parallel.combine_partials(parts, combine=lambda x: torch.from_numpy(oracle.combine_ct(x.numpy())))
    frame = parallel.gather_frames(band, H)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_plane_sharded_exchange_matches_sequential(world, tmp_path):
    sys.path.insert(0, REPO)
    from oracle import oracle
    out = str(tmp_path / "frame.npy")
    mp.spawn(_plane_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    mpi, homs = _case()
    want = oracle.render(mpi, homs)
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)


def _empty_shard_worker(rank, world, port, H, W, P, out_path):
    """The product's render_plane_sharded / render_view_sharded with more ranks than planes,
    rows or views (such a rank used to raise while the others waited in the
    collective).  The per-rank kernels are replaced by the oracle (CPU tensors)."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_vision_amd import _lib, parallel
    from oracle import oracle
    mpi, homs = _case(H, W, P)
    V = mpi.shape[0]
    p0, p1 = parallel.shard_range(P, rank, world)
    packed = torch.zeros(_lib.packed_shape(H, W, p1 - p0))
    packed[:, 2:2 + H, 2:2 + W] = torch.from_numpy(mpi[0, :, :, p0:p1]).permute(2, 0, 1, 3)
    local = np.ascontiguousarray(mpi[:, :, :, p0:p1])
    frame = parallel.render_plane_sharded(
        packed, torch.from_numpy(np.ascontiguousarray(homs[:, p0:p1])), H,
        render_ct=lambda pk, h, back: torch.from_numpy(oracle.render_ct(local, h.numpy(), 0, p1 - p0, back)),
        combine=lambda x: torch.from_numpy(oracle.combine_ct(x.numpy())))
    # view sharding with more ranks than views: 2 views over `world` ranks
    full_pk = torch.zeros(_lib.packed_shape(H, W, P))
    full_pk[:, 2:2 + H, 2:2 + W] = torch.from_numpy(mpi[0]).permute(2, 0, 1, 3)
    views = parallel.render_view_sharded(
        full_pk, torch.from_numpy(homs), gather=True,
        render=lambda pk, h: torch.from_numpy(oracle.render(np.ascontiguousarray(mpi[:h.shape[0]]), h.numpy())))
    if rank == 0:
        np.save(out_path, frame.numpy())
        np.save(out_path + ".views.npy", views.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,P", [(3, 9, 13, 2), (3, 2, 11, 5), (4, 3, 6, 2)])
def test_more_ranks_than_planes_rows_views(world, H, W, P, tmp_path):
    """Ranks with no planes contribute the identity partial, ranks with no rows an empty
    band, ranks with no views an empty shard: the job completes and rank 0's frames match
    the sequential render (1e-5 plane-sharded; views bit-exact up to the view order)."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    out = str(tmp_path / "frame.npy")
    mp.spawn(_empty_shard_worker, args=(world, _free_port(), H, W, P, out), nprocs=world, join=True)
    mpi, homs = _case(H, W, P)
    want = oracle.render(mpi, homs)
    np.testing.assert_allclose(np.load(out), want, rtol=0, atol=1e-5)
    np.testing.assert_array_equal(np.load(out + ".views.npy"), want)


def _pipelined_worker(rank, world, port, H, W, P, out_path):
    """render_plane_sharded's pipelined path (bands rendered one at a time, each band's pair
    exchange posted as soon as it is rendered) with oracle row bands standing in for
    mpiv_render_packed_ct_rows: the same frame, bit for bit, as the one-shot all-to-all path."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_vision_amd import _lib, parallel
    from oracle import oracle
    mpi, homs = _case(H, W, P)
    p0, p1 = parallel.shard_range(P, rank, world)
    packed = torch.zeros(_lib.packed_shape(H, W, p1 - p0))
    local = np.ascontiguousarray(mpi[:, :, :, p0:p1])
    full = torch.from_numpy(oracle.render_ct(local, homs[:, p0:p1], 0, p1 - p0, rank == 0)) if p1 > p0 else None
    bands_done = []

    def rows(pk, h, back, y0, y1, out):
        bands_done.append((y0, y1))
        out[:, y0:y1] = full[:, y0:y1]
        return out
    comb = lambda x: torch.from_numpy(oracle.combine_ct(x.numpy()))  # noqa: E731
    hl = torch.from_numpy(np.ascontiguousarray(homs[:, p0:p1]))
    stats = {}
    # forced on: short frames (H < world, empty bands) take the one-shot path by default
    got = parallel.render_plane_sharded(packed, hl, H, render_rows=rows, combine=comb, stats=stats, pipelined=True)
    one = parallel.render_plane_sharded(packed, hl, H, render_ct=lambda pk, h, back: full, combine=comb,
                                        pipelined=False) if p1 > p0 else \
        parallel.render_plane_sharded(packed, hl, H, combine=comb, pipelined=False)
    # every non-empty band of this rank rendered exactly once, its own band last
    bb = parallel.band_bounds(H, world)
    if p1 > p0:
        want_order = [bb[(rank + s) % world] for s in range(1, world)] + [bb[rank]]
        assert bands_done == [b for b in want_order if b[1] > b[0]], (rank, bands_done)
    assert stats["steps"] == world - 1
    if rank == 0:
        np.save(out_path, got.numpy())
        np.save(out_path + ".one.npy", one.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,P", [(2, 37, 53, 11), (3, 37, 53, 11), (4, 3, 6, 2), (3, 2, 11, 5),
                                         # the driver's 8-GPU node: config 5's 2160-row frame cut into
                                         # 8 bands of 270 rows, and a frame shorter than the world
                                         (8, 2160, 5, 16), (8, 5, 6, 3)])
def test_plane_sharded_pipelined_equals_one_shot(world, H, W, P, tmp_path):
    """The pipelined band exchange (SURVEY §8e "pipeline bands to overlap") on gloo at world
    2, 3, 4 and 8 (incl. ranks with no planes and with no rows): bit-identical to the one-shot
    all-to-all path, and within 1e-5 of the sequential render."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    out = str(tmp_path / "frame.npy")
    mp.spawn(_pipelined_worker, args=(world, _free_port(), H, W, P, out), nprocs=world, join=True)
    got, one = np.load(out), np.load(out + ".one.npy")
    assert np.array_equal(got.view(np.uint32), one.view(np.uint32))
    mpi, homs = _case(H, W, P)
    np.testing.assert_allclose(got, oracle.render(mpi, homs), rtol=0, atol=1e-5)


def test_pipeline_default_needs_every_band_non_empty():
    sys.path.insert(0, REPO)
    from mpi_vision_amd import parallel
    assert parallel.pipeline_by_default(8, 2160, 4096)
    assert parallel.pipeline_by_default(2, 2, 2)
    assert not parallel.pipeline_by_default(1, 2160, 4096)
    assert not parallel.pipeline_by_default(4, 3, 6)   # one rank's band would be empty
    assert not parallel.pipeline_by_default(3, 37, 1)


def test_shard_ranges_cover_exactly():
    sys.path.insert(0, REPO)
    from mpi_vision_amd import parallel
    for n in (1, 7, 128, 256, 1000):
        for world in (1, 2, 3, 8):
            ranges = [parallel.shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [e - b for b, e in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_ct_partials_single_process_reassociation():
    """Combining 1..P single-plane partials equals the sequential render within 1e-5."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    mpi, homs = _case()
    P = mpi.shape[3]
    want = oracle.render(mpi, homs)
    for cuts in ([0, P], [0, 4, P], list(range(P + 1))):
        parts = np.stack([oracle.render_ct(mpi, homs, a, b, back=(a == 0)) for a, b in zip(cuts[:-1], cuts[1:])])
        np.testing.assert_allclose(oracle.combine_ct(parts), want, rtol=0, atol=1e-5)
        if len(cuts) == 2:
            assert np.array_equal(oracle.combine_ct(parts), want)


def _plane_worker_gpu(rank, world, port, out_path, shape=(37, 53, 11)):
    """One rank of the plane-sharded render with the HIP kernels (every rank on cuda:0,
    gloo collectives staged through host memory): packed local planes -> (C, T) partial
    (mpiv_render_packed_ct) -> band all-to-all -> ordered combine (mpiv_combine_ct) ->
    frame gather."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_vision_amd import _lib, parallel
    dev = torch.device("cuda:0")
    mpi, homs = _case(*shape)
    V, H, W, P, _ = mpi.shape
    p0, p1 = parallel.shard_range(P, rank, world)
    if p1 > p0:
        packed = _lib.pack_planes(torch.from_numpy(np.ascontiguousarray(mpi[0, :, :, p0:p1])).to(dev))
    else:  # more ranks than planes: this rank owns none
        packed = torch.zeros(_lib.packed_shape(H, W, 0), device=dev)
    homs_local = torch.from_numpy(np.ascontiguousarray(homs[:, p0:p1])).to(dev)
    frame = parallel.render_plane_sharded(packed, homs_local, H)
    if rank == 0:
        np.save(out_path, frame.cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,shape", [(2, (37, 53, 11)), (3, (37, 53, 11)), (3, (2, 11, 5)), (4, (3, 6, 2))])
def test_plane_sharded_hip_ranks_match_sequential(world, shape, tmp_path):
    """The whole plane-sharded path on the GPU kernels, world 2 and 3 (ranks share one
    device; the driver's 8-GPU node runs the same code over RCCL), incl. more ranks than
    planes / rows: within 1e-5 of the sequential oracle render."""
    sys.path.insert(0, REPO)
    from oracle import oracle
    out = str(tmp_path / "frame.npy")
    mp.spawn(_plane_worker_gpu, args=(world, _free_port(), out, shape), nprocs=world, join=True)
    got = np.load(out)
    mpi, homs = _case(*shape)
    want = oracle.render(mpi, homs)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)


def _view_gather_worker(rank, world, port, n_views, out_path):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_vision_amd import parallel
    sl = parallel.view_shard(n_views, rank, world)
    # frame v is filled with v (+ a per-pixel ramp) so order and trimming are checked
    ramp = torch.arange(4 * 5 * 3, dtype=torch.float32).reshape(4, 5, 3) / 1000.0
    frames = torch.stack([ramp + v for v in range(sl.start, sl.stop)]) if sl.stop > sl.start \
        else torch.zeros((0, 4, 5, 3))
    got = parallel.gather_view_frames(frames, n_views)
    if rank == 0:
        np.save(out_path, got.numpy())
    else:
        assert got is None
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_views", [(2, 7), (3, 7), (3, 2), (8, 13), (8, 5)])
def test_view_sharded_gather_uneven(world, n_views, tmp_path):
    """View sharding's final frame gather with uneven shards (incl. a rank
    holding no views): rank 0 gets every frame, in camera-path order."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_view_gather_worker, args=(world, _free_port(), n_views, out), nprocs=world, join=True)
    got = np.load(out)
    ramp = np.arange(60, dtype=np.float32).reshape(4, 5, 3) / np.float32(1000.0)
    want = np.stack([ramp + np.float32(v) for v in range(n_views)])
    np.testing.assert_array_equal(got, want)


def _view_worker_gpu(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpi_vision_amd import _host, _lib, configs, parallel
    dev = torch.device("cuda:0")
    H, W, P, V = 37, 53, 11, 5
    mpi = configs.synthetic_mpi(1, H, W, P, 5)
    K = configs.f32([configs.intrinsics_matrix(50.0, 52.0, 26.0, 18.0)] * V)
    poses = configs.f32([configs.pose_from(configs.rot_y(1.5 - v), (0.05 * v, -0.02, 0.03)) for v in range(V)])
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 20, P)), K, V).to(dev)
    packed = _lib.pack_planes(mpi[0].to(dev))
    frames = parallel.render_view_sharded(packed, homs, gather=True)
    if rank == 0:
        np.save(out_path, frames.cpu().numpy())
        np.save(out_path + ".seq.npy", _lib.render_packed(packed, homs).cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_view_sharded_hip_ranks_gather_bit_exact(world, tmp_path):
    """View-sharded render on the HIP kernels (5 views over 2 / 3 ranks sharing one device)
    with the final frame gather: bit-identical to one launch of all views."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_view_worker_gpu, args=(world, _free_port(), out), nprocs=world, join=True)
    np.testing.assert_array_equal(np.load(out), np.load(out + ".seq.npy"))


def _rccl_worker(rank, world, port, out_path):
    """Both sharded paths with the device collectives on RCCL ("nccl"): world 1 is the
    most a one-GPU box allows (RCCL refuses two ranks on one device: "Duplicate GPU
    detected"), so this checks the RCCL calls themselves -- all_to_all_single and gather
    on device tensors, no host staging -- that the 8-GPU node runs at world 8."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from mpi_vision_amd import _host, _lib, configs, parallel
    assert dist.get_backend() == "nccl"
    H, W, P, V = 37, 53, 11, 5
    mpi = configs.synthetic_mpi(1, H, W, P, 5)
    K = configs.f32([configs.intrinsics_matrix(50.0, 52.0, 26.0, 18.0)] * V)
    poses = configs.f32([configs.pose_from(configs.rot_y(1.5 - v), (0.05 * v, -0.02, 0.03)) for v in range(V)])
    homs = _host.render_homographies(poses, configs.f32(configs.inv_depths(1, 20, P)), K, V).to(dev)
    packed = _lib.pack_planes(mpi[0].to(dev))
    frames = parallel.render_view_sharded(packed, homs, gather=True)
    p0, p1 = parallel.shard_range(P, rank, world)
    local = _lib.pack_planes(mpi[0, :, :, p0:p1].contiguous().to(dev))
    frame = parallel.render_plane_sharded(local, homs[:1, p0:p1].contiguous(), H)
    if rank == 0:
        assert frames.is_cuda and frame.is_cuda
        np.save(out_path, frames.cpu().numpy())
        np.save(out_path + ".plane.npy", frame.cpu().numpy())
        np.save(out_path + ".seq.npy", _lib.render_packed(packed, homs).cpu().numpy())
    # the pipelined band exchange's own RCCL calls: this rank plays 4 band
    # ranks against itself (every P2P op goes to rank 0: a self send / receive pair per step), so
    # render_plane_sharded_pipelined posts its batch_isend_irecv between the per-band row renders
    # exactly as at world 4; 2 views make every send a .contiguous() temporary.  Received band j
    # at step s is this rank's band s, so the combine sees bands 0, 3, 2, 1 in that order.
    G, H2 = 4, 36
    packed2 = _lib.pack_planes(configs.synthetic_mpi(1, H2, W, P, 6)[0].to(dev))
    homs2 = homs[:2].contiguous()
    stats = {}
    got = parallel.render_plane_sharded_pipelined(packed2, homs2, H2, world=(G, 0), peer=lambda r: 0, stats=stats)
    ct = _lib.render_packed_ct(packed2, homs2, back=True)
    bh = H2 // G
    parts = torch.stack([ct[:, k * bh:(k + 1) * bh] for k in (0, 3, 2, 1)])
    if rank == 0:
        np.save(out_path + ".pipe.npy", got.cpu().numpy())
        np.save(out_path + ".pipe_want.npy", _lib.combine_ct(parts.contiguous()).cpu().numpy())
        np.save(out_path + ".pipe_sent.npy", np.array([stats["bytes_sent"], stats["steps"]]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_paths_over_rccl_world1(tmp_path):
    """View- and plane-sharded renders through RCCL device collectives (world 1 on the
    one-GPU box): bit-identical to one launch of all views / all planes."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_rccl_worker, args=(1, _free_port(), out), nprocs=1, join=True)
    seq = np.load(out + ".seq.npy")
    np.testing.assert_array_equal(np.load(out), seq)
    np.testing.assert_array_equal(np.load(out + ".plane.npy"), seq[:1])
    np.testing.assert_array_equal(np.load(out + ".pipe.npy"), np.load(out + ".pipe_want.npy"))
    assert list(np.load(out + ".pipe_sent.npy")) == [3 * 2 * 9 * 53 * 4 * 4, 3]

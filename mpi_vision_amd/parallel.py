"""Multi-GPU sharding of the MPI render.  One process per GPU,
torch.distributed over RCCL ("nccl") on the box, gloo in CPU tests.

* View sharding (configs 2/4): the camera path is split into contiguous pose
  ranges, every rank renders its views from its own MPI replica -- no collective on
  the data path; frames stay in HBM unless `gather_frames` is asked for.

* Plane sharding (config 5): rank g owns planes [g*P/G, (g+1)*P/G), back to front,
  and renders the partial (C, T) of its range (`mpiv_render_packed_ct`).  The
  over-operator (Cf, Tf) o (Cb, Tb) = (Cf + Tf*Cb, Tf*Tb) is associative but NOT
  commutative and RCCL has no custom reduction op, so the combine is an ordered
  exchange instead of an all-reduce:
      1. the frame is cut into G row bands; one all_to_all (RCCL point-to-point
         over xGMI: every GPU sends G-1 bands and receives G-1 bands at once, one
         per link, instead of a ring that is bound by one link) leaves rank k with
         band k of every shard's partial, in plane order (source rank order);
      2. rank k combines them back-to-front with `mpiv_combine_ct`;
      3. the RGB bands are gathered to the destination rank.
  Parity: reassociating the over-operator across G ranges moves results by ~1e-7
  (SURVEY.md §8e measured 2.4e-7 over 8 ranges of 256 planes); the tests hold it to
  1e-5 against the single-GPU sequential render.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Balanced contiguous split of n items: rank's [begin, end)."""
    q, r = divmod(n, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def band_bounds(height: int, world: int) -> list[tuple[int, int]]:
    return [shard_range(height, k, world) for k in range(world)]


def _world(group):
    return dist.get_world_size(group), dist.get_rank(group)


def _staged(t: torch.Tensor, group) -> bool:
    """gloo collectives take host tensors: device tensors are staged through host memory
    (a rehearsal of the multi-rank path on one device; RCCL moves device tensors directly)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def exchange_bands(ct: torch.Tensor, group=None) -> torch.Tensor:
    """all_to_all of row bands.

    ct: this rank's partial [V, H, W, 4] (C, T) for its plane range.
    Returns [G, V, bh, W, 4]: band `rank` of every rank's partial, indexed by source
    rank (= plane order, back first), padded to the tallest band bh."""
    G, rank = _world(group)
    V, H, W, C = ct.shape
    bands = band_bounds(H, G)
    bh = max(e - b for b, e in bands)
    if V == 1 and H % G == 0 and ct.is_contiguous():
        send = ct.view(G, 1, bh, W, C)  # the bands are already consecutive row ranges: no copy
    else:
        send = ct.new_zeros((G, V, bh, W, C))
        for k, (b, e) in enumerate(bands):
            send[k, :, : e - b] = ct[:, b:e]
    if _staged(send, group):
        send_h = send.cpu()
        recv_h = torch.empty_like(send_h)
        dist.all_to_all_single(recv_h, send_h, group=group)
        recv = recv_h.to(send.device)
    else:
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=group)
    b, e = bands[rank]
    return recv[:, :, : e - b]


def gather_frames(band: torch.Tensor, height: int, group=None, dst: int = 0) -> Optional[torch.Tensor]:
    """Gather RGB row bands [V, bh_k, W, 3] (band k on rank k) into [V, H, W, 3] on dst."""
    G, rank = _world(group)
    bands = band_bounds(height, G)
    bh = max(e - b for b, e in bands)
    V, h, W, C = band.shape
    if h == bh and band.is_contiguous():
        padded = band
    else:
        padded = band.new_zeros((V, bh, W, C))
        padded[:, :h] = band
    dev = padded.device
    if _staged(padded, group):
        padded = padded.cpu()
    gathered = [torch.empty_like(padded) for _ in range(G)] if rank == dst else None
    dist.gather(padded, gathered, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([g[:, : e - b] for g, (b, e) in zip(gathered, bands)], dim=1).to(dev)


def combine_partials(parts: torch.Tensor,
                     combine: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> torch.Tensor:
    """Ordered back-to-front over-combine of [G, ...,4] partials -> [..., 3] (HIP kernel).
    An empty band (a frame with fewer rows than ranks) combines to an empty band."""
    if parts[0].numel() == 0:
        return parts.new_empty(tuple(parts.shape[1:-1]) + (3,))
    if combine is None:
        from . import _lib
        combine = _lib.combine_ct
    return combine(parts)


def identity_partial(views: int, height: int, width: int, like: torch.Tensor) -> torch.Tensor:
    """The (C, T) partial of an empty plane range, (0, 1): the over-operator's identity, so a
    rank that owns no planes (P < ranks) leaves the combined frame unchanged."""
    ct = like.new_zeros((views, height, width, 4))
    ct[..., 3] = 1.0
    return ct


def pipeline_by_default(world: int, height: int, width: int) -> bool:
    """The band pipeline is the default when there is more than one rank and every row band is
    non-empty (height >= world), so every rank posts a P2P batch at every step (with
    RCCL, a rank that skips a group's first P2P batch while the others post is undefined).
    Shorter frames take the one-shot all-to-all (gloo tests still drive the pipeline on them)."""
    return world > 1 and height >= world and width >= 2


def render_plane_sharded(packed_local: torch.Tensor, homs_local: torch.Tensor, height: int, group=None,
                         dst: int = 0, render_ct: Optional[Callable] = None,
                         combine: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
                         render_rows: Optional[Callable] = None, pipelined: Optional[bool] = None,
                         stats: Optional[dict] = None) -> Optional[torch.Tensor]:
    """Plane-sharded render of V views.

    packed_local: this rank's planes, packed [P_local, H+4, W+4, 4] (_lib.pack_planes) (rank 0 holds the
    back-most range, which contains the reference's plane 0); homs_local
    [V, P_local, 9].  P_local may be 0 (more ranks than planes): that rank contributes the
    identity partial.  Returns the final frames [V, H, W, 3] on dst, None elsewhere.

    pipelined (default on the GPU path: pipeline_by_default): the partial is rendered band by band and each band leaves for its rank as soon as it
    is rendered, overlapping the next band's render (render_plane_sharded_pipelined); else one
    render, one all-to-all.  render_ct / render_rows / combine replace the HIP kernels (CPU
    tests of the exchange logic only)."""
    from . import _lib
    G, rank = _world(group)
    V = homs_local.shape[0]
    width = packed_local.shape[2] - 2 * _lib.PAD
    if pipelined is None:
        pipelined = pipeline_by_default(G, height, width) and (render_rows is not None or render_ct is None)
    if pipelined:
        return render_plane_sharded_pipelined(packed_local, homs_local, height, group, dst, render_rows, combine,
                                              stats)
    if packed_local.shape[0] == 0:
        ct = identity_partial(V, height, width, packed_local)
    else:
        ct = (render_ct or _lib.render_packed_ct)(packed_local, homs_local, back=(rank == 0))
    parts = exchange_bands(ct, group)
    band = combine_partials(parts, combine)
    return gather_frames(band, height, group, dst)


def render_plane_sharded_pipelined(packed_local: torch.Tensor, homs_local: torch.Tensor, height: int, group=None,
                                   dst: int = 0, render_rows: Optional[Callable] = None,
                                   combine: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
                                   stats: Optional[dict] = None, world: Optional[tuple[int, int]] = None,
                                   peer: Optional[Callable[[int], int]] = None) -> Optional[torch.Tensor]:
    """render_plane_sharded with the band exchange overlapped with the render (SURVEY.md §8e
    "pipeline bands to overlap").  G - 1 steps: at step s rank r renders row band k = r + s
    (mod G) of its partial (mpiv_render_packed_ct_rows, one launch) and posts one batched
    pair exchange -- band k to rank k, band r from rank r - s -- then goes on to the next band
    while the exchange runs (RCCL's stream waits only for the work enqueued before the post).
    Every rank walks the steps in the same order, so each step's sends and receives pair up.
    Its own band r is rendered last and combined with the received ones in plane (source rank)
    order (mpiv_combine_ct, as the one-shot path), then the RGB bands are gathered.
    stats (optional): filled with the bytes this rank sent and the steps posted.
    world / peer (tests only): the (G, rank) the band schedule uses and the process-group rank a
    band rank's P2P ops go to -- a world-1 RCCL test plays G band ranks against itself (self
    send / receive) to run this function's posting on the device; the frames are then not a
    render of the MPI, and gather_frames is skipped (the band is returned).

    The send tensors (a view of ct, or its contiguous copy when V > 1) are kept referenced until
    every exchange has completed (wait()), so the caching allocator cannot hand their memory to
    the next band's render while RCCL still reads it."""
    from . import _lib
    G, rank = _world(group) if world is None else world
    to = peer or (lambda r: r)
    V = homs_local.shape[0]
    width = packed_local.shape[2] - 2 * _lib.PAD
    bands = band_bounds(height, G)
    b_r, e_r = bands[rank]
    empty = packed_local.shape[0] == 0
    ct = identity_partial(V, height, width, packed_local) if empty else \
        packed_local.new_empty((V, height, width, 4))
    rows = render_rows or _lib.render_packed_ct_rows
    staged = _staged(ct, group)
    recv = ct.new_empty((G, V, e_r - b_r, width, 4))  # band r of every rank's partial, by source rank
    host_recv = {}
    works, keep, sent = [], [], 0

    def render_band(k):
        b, e = bands[k]
        if e > b and not empty:
            rows(packed_local, homs_local, rank == 0, b, e, ct)

    for s in range(1, G):
        k, j = (rank + s) % G, (rank - s) % G  # this step's destination and source
        render_band(k)
        ops = []
        b, e = bands[k]
        if e > b:
            snd = ct[:, b:e]
            snd = snd.contiguous() if not snd.is_contiguous() else snd
            if staged:
                snd = snd.cpu()
            keep.append(snd)
            ops.append(dist.P2POp(dist.isend, snd, to(k), group))
            sent += snd.numel() * snd.element_size()
        if e_r > b_r:
            rb = recv[j]
            if staged:
                rb = host_recv[j] = torch.empty(tuple(rb.shape), dtype=rb.dtype)
            ops.append(dist.P2POp(dist.irecv, rb, to(j), group))
        if ops:
            works += dist.batch_isend_irecv(ops)
    render_band(rank)
    recv[rank] = ct[:, b_r:e_r]
    for w in works:
        w.wait()
    keep.clear()  # the exchanges are complete (on RCCL: the current stream now waits for them)
    for j, hb in host_recv.items():
        recv[j].copy_(hb)
    if stats is not None:
        stats.update(bytes_sent=sent, steps=G - 1)
    band = combine_partials(recv, combine)
    return band if world is not None else gather_frames(band, height, group, dst)


def view_shard(n_views: int, rank: int, world: int) -> slice:
    b, e = shard_range(n_views, rank, world)
    return slice(b, e)


def gather_view_frames(frames: torch.Tensor, n_views: int, group=None, dst: int = 0) -> Optional[torch.Tensor]:
    """The view-sharded path's one optional collective (SURVEY.md §8e "final frame
    gather"): rank k's frames [v_k, H, W, 3] of poses view_shard(n_views, k, G) -> the
    whole camera path [n_views, H, W, 3] on dst (None elsewhere).  Shards may be uneven
    (n_views % G != 0): each is padded to the largest for one gather and trimmed."""
    G, rank = _world(group)
    sizes = [e - b for b, e in (shard_range(n_views, k, G) for k in range(G))]
    if frames.shape[0] != sizes[rank]:
        raise RuntimeError(f"gather_view_frames: rank {rank} holds {frames.shape[0]} views, "
                           f"its shard has {sizes[rank]}")
    padded = frames.new_zeros((max(sizes),) + tuple(frames.shape[1:]))
    padded[: sizes[rank]] = frames
    dev = padded.device
    if _staged(padded, group):
        padded = padded.cpu()
    gathered = [torch.empty_like(padded) for _ in range(G)] if rank == dst else None
    dist.gather(padded, gathered, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([g[:n] for g, n in zip(gathered, sizes)], dim=0).to(dev)


def render_view_sharded(packed: torch.Tensor, homs_all: torch.Tensor, group=None, gather: bool = False,
                        dst: int = 0, render: Optional[Callable] = None) -> Optional[torch.Tensor]:
    """This rank's frames of a view-sharded camera path (no collective); with `gather`,
    the whole path's frames on dst (gather_view_frames) and None elsewhere.  A rank whose
    shard is empty (fewer views than ranks) renders nothing and still joins the gather.
    render replaces the HIP kernel (CPU tests of the sharding logic only)."""
    from . import _lib
    G, rank = _world(group)
    sl = view_shard(homs_all.shape[0], rank, G)
    hv = homs_all[sl]
    if hv.shape[0] == 0:
        H, W = packed.shape[1] - 2 * _lib.PAD, packed.shape[2] - 2 * _lib.PAD
        frames = packed.new_empty((0, H, W, 3))
    else:
        frames = (render or _lib.render_packed)(packed, hv)
    return gather_view_frames(frames, homs_all.shape[0], group, dst) if gather else frames

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


def render_plane_sharded(packed_local: torch.Tensor, homs_local: torch.Tensor, height: int, group=None,
                         dst: int = 0, render_ct: Optional[Callable] = None,
                         combine: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> Optional[torch.Tensor]:
    """Plane-sharded render of V views.

    packed_local: this rank's planes, packed [P_local, H+4, W+4, 4] (_lib.pack_planes) (rank 0 holds the
    back-most range, which contains the reference's plane 0); homs_local
    [V, P_local, 9].  P_local may be 0 (more ranks than planes): that rank contributes the
    identity partial.  Returns the final frames [V, H, W, 3] on dst, None elsewhere.
    render_ct / combine replace the HIP kernels (CPU tests of the exchange logic only)."""
    from . import _lib
    G, rank = _world(group)
    V = homs_local.shape[0]
    width = packed_local.shape[2] - 2 * _lib.PAD
    if packed_local.shape[0] == 0:
        ct = identity_partial(V, height, width, packed_local)
    else:
        ct = (render_ct or _lib.render_packed_ct)(packed_local, homs_local, back=(rank == 0))
    parts = exchange_bands(ct, group)
    band = combine_partials(parts, combine)
    return gather_frames(band, height, group, dst)


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

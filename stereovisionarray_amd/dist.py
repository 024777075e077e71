"""Multi-GPU plumbing for independent stereo units.

One process per GPU.  Units (camera pairs, frames) are independent: unit i is
matched by rank i mod N with no data-path collective; the only exchange is the
gather of the final u16 disparity maps to the root (RCCL over xGMI when the
process group backend is "nccl"; gloo in the CPU tests).  This module is
torch.distributed plumbing only -- every disparity and fusion computation runs
in libsva.so kernels.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(n_units: int, rank: int, world: int) -> list[int]:
    """Units owned by `rank`: i with i mod world == rank (round-robin)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return list(range(rank, n_units, world))


def slots(n_units: int, world: int) -> int:
    """Per-rank slot count used by the gather (ceil(n_units / world))."""
    return (n_units + world - 1) // world


def gather_maps(local: torch.Tensor, n_units: int, dst: int = 0,
                group=None) -> torch.Tensor | None:
    """Gather per-rank maps [n_local, H, W] to `dst`, returned there as
    [n_units, H, W] in unit order (None elsewhere).

    Ranks own unequal unit counts when world does not divide n_units; every
    rank sends ceil(n_units/world) slots (padding unused ones) so one
    fixed-size gather serves all ranks.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = shard(n_units, rank, world)
    if local.shape[0] != len(mine):
        raise ValueError(f"rank {rank} owns {len(mine)} units, got {local.shape[0]} maps")
    k = slots(n_units, world)
    shape, dtype = tuple(local.shape[1:]), local.dtype
    # ship raw bytes: every backend gathers uint8 (gloo rejects e.g. int16)
    row = local.element_size()
    for n in shape:
        row *= n
    local = local.contiguous().view(torch.uint8).reshape(local.shape[0], row)
    send = local
    if local.shape[0] < k:
        pad = torch.zeros((k - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        send = torch.cat([local, pad], 0)
    if rank == dst:
        bufs = [torch.empty_like(send) for _ in range(world)]
        dist.gather(send.contiguous(), bufs, dst=dst, group=group)
        out = torch.empty((n_units,) + tuple(local.shape[1:]), dtype=torch.uint8,
                          device=local.device)
        for r in range(world):
            for j, u in enumerate(shard(n_units, r, world)):
                out[u] = bufs[r][j]
        return out.view(dtype).reshape((n_units,) + shape)
    dist.gather(send.contiguous(), None, dst=dst, group=group)
    return None


def _row_bytes(t: torch.Tensor) -> int:
    row = t.element_size()
    for n in t.shape[1:]:
        row *= n
    return row


def checksums(maps: torch.Tensor) -> torch.Tensor:
    """Per-unit checksum of maps [n, ...] as int64 [n]: a position-weighted
    byte sum (weights 1..251 repeating), so swapped units, shifted rows and
    single-byte errors all change it.  Runs on the maps' device."""
    n, row = maps.shape[0], _row_bytes(maps)
    b = maps.contiguous().view(torch.uint8).reshape(n, row).to(torch.int64)
    w = torch.arange(b.shape[1], device=b.device, dtype=torch.int64) % 251 + 1
    return (b * w).sum(1)


def gather_maps_checked(local: torch.Tensor, n_units: int, dst: int = 0, group=None):
    """gather_maps with a per-unit checksum computed by the owning rank and
    shipped with its map: on `dst` returns (maps [n_units, ...], ok) where ok
    says every received map matches the checksum its owner computed before
    sending; (None, True) elsewhere.  Used once per run by bench.py to check
    the multi-rank exchange (the timed steps use plain gather_maps)."""
    n = local.shape[0]
    row = local.contiguous().view(torch.uint8).reshape(n, _row_bytes(local))
    ck = checksums(local).view(torch.uint8).reshape(n, 8)
    packed = torch.cat([row, ck], 1)
    out = gather_maps(packed, n_units, dst=dst, group=group)
    if out is None:
        return None, True
    maps = out[:, :-8].contiguous()
    sent = out[:, -8:].contiguous().view(torch.int64).reshape(n_units)
    shape = (n_units,) + tuple(local.shape[1:])
    maps = maps.view(local.dtype).reshape(shape)
    ok = bool(torch.equal(checksums(maps), sent))
    return maps, ok

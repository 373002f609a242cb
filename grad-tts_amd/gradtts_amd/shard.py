"""Utterance sharding across ranks (one process per GPU, torch.distributed over RCCL / gloo).

The decoder path has no cross-utterance dependency: every utterance of a batch is decoded
independently (GroupNorm and attention statistics are per utterance, and the HIP path is
batch-invariant -- tests/test_decoder_gpu.py). Multi-GPU therefore means data-parallel shards of
utterances with no collective inside the decode; the only exchange is gathering the finished mels
where the caller wants them in one place.

  shard_bounds(n, rank, world)       contiguous split of n utterances, sizes differ by at most one
  shard(x, rank, world)              this rank's rows of a [n, ...] tensor
  gather_shards(y, n, world)         all ranks' shards reassembled in utterance order (all_gather)
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard(x: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    lo, hi = shard_bounds(x.shape[0], rank, world)
    return x[lo:hi].contiguous()


def gather_shards(y: torch.Tensor, n: int, world: int, group=None) -> torch.Tensor:
    """Concatenate every rank's shard (rows lo:hi of the global batch) in rank order.

    Shards are padded to the largest shard size so that one all_gather moves equal-sized buffers
    (RCCL and gloo both require that), then trimmed."""
    if world == 1:
        return y
    sizes = [shard_bounds(n, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    buf = y.new_zeros((cap,) + tuple(y.shape[1:]))
    buf[: y.shape[0]] = y
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[: hi - lo] for p, (lo, hi) in zip(parts, sizes)], dim=0)

"""Multi-GPU plumbing for the vocoder: one process per GPU, utterances sharded
over ranks, weights broadcast once.

The reference is single-process; utterances are independent
(no op mixes batch items), so the only collective on this
path is ONE broadcast of the flattened weights from rank 0 at start-up —
``torch.distributed`` backend "nccl" is RCCL over xGMI on MI355X, "gloo" on
CPU for the tests.  Steady state has no collective at all.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
import torch.distributed as dist


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of `total` items for `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def balance_by_length(lengths: List[int], world: int) -> List[List[int]]:
    """Greedy longest-first assignment of variable-length utterances to ranks,
    balancing the sum of frames."""
    order = sorted(range(len(lengths)), key=lambda i: -lengths[i])
    load = [0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        out[r].append(i)
        load[r] += lengths[i]
    return [sorted(o) for o in out]


def broadcast_state_dict(sd: Dict[str, torch.Tensor] | None, spec: List[Tuple[str, tuple]],
                         device: torch.device, src: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Broadcast fp32 tensors named/shaped by `spec` from `src` as ONE flat buffer
    (one large collective instead of one per tensor).  `sd` is only read on src."""
    numel = [int(torch.Size(s).numel()) for _, s in spec]
    flat = torch.empty(sum(numel), dtype=torch.float32, device=device)
    if dist.get_rank() == src:
        off = 0
        for (k, _), n in zip(spec, numel):
            flat[off:off + n].copy_(torch.as_tensor(sd[k]).reshape(-1))
            off += n
    dist.broadcast(flat, src)
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    off = 0
    for (k, s), n in zip(spec, numel):
        out[k] = flat[off:off + n].view(s)
        off += n
    return out

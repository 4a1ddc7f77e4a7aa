"""Multi-GPU plumbing for the vocoder: one process per GPU, utterances sharded
over ranks, weights broadcast once, wavs gathered to one rank.

The reference is single-process; utterances are independent
(no op mixes batch items), so the collectives on this path are
ONE broadcast of the flattened weights from rank 0 at start-up and, for the
product call :func:`vocode_sharded`, one gather of every rank's (padded) wavs to
the gathering rank — ``torch.distributed`` backend "nccl" is RCCL over xGMI on
MI355X, "gloo" on CPU for the tests.  The steady-state forward itself has no
collective.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

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
    balancing the sum of frames.  Deterministic: every
    rank computes the same assignment from the same lengths."""
    order = sorted(range(len(lengths)), key=lambda i: (-lengths[i], i))
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


def _coll_device(device: torch.device, group) -> torch.device:
    """Where collective buffers live: the GPU for RCCL, the host for gloo."""
    return device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _broadcast_batch(mel: Optional[torch.Tensor], lengths: Optional[Sequence[int]], src: int,
                     device: torch.device, group):
    """Rank `src`'s (mel, lengths) on every rank: shape / lengths as one small
    int64 broadcast, then the mel as one fp32 broadcast."""
    cdev = _coll_device(device, group)
    me = dist.get_rank(group)
    gsrc = src if group is None else dist.get_global_rank(group, src)  # broadcast: global rank
    head = torch.zeros(4, dtype=torch.int64, device=cdev)
    if me == src:
        if mel is None or mel.dim() != 3:
            raise RuntimeError("vocode_sharded: rank src must pass a 3-D mel batch")
        head[:3] = torch.tensor(list(mel.shape), dtype=torch.int64)
        head[3] = 0 if lengths is None else 1
    dist.broadcast(head, gsrc, group=group)
    shape = [int(v) for v in head[:3].tolist()]
    lens_t = torch.zeros(shape[0], dtype=torch.int64, device=cdev)
    if int(head[3]):
        if me == src:
            lens_t.copy_(torch.as_tensor([int(x) for x in lengths], dtype=torch.int64))
        dist.broadcast(lens_t, gsrc, group=group)
        lens = [int(v) for v in lens_t.tolist()]
    else:
        lens = None
    buf = (mel.detach().to(device=cdev, dtype=torch.float32).contiguous() if me == src
           else torch.empty(shape, dtype=torch.float32, device=cdev))
    dist.broadcast(buf, gsrc, group=group)
    return buf, lens


def vocode_sharded(gen, mel: Optional[torch.Tensor], lengths: Optional[Sequence[int]] = None, *,
                   mel_layout: str = "bct", dst: Optional[int] = 0, src: Optional[int] = None,
                   device: Optional[torch.device] = None, group=None):
    """Vocode one batch of utterances across the ranks of a process group.

    Every rank calls this with the same arguments (collective call).  The batch —
    ``mel`` [B, n_mels, T] (``mel_layout="bct"``) or the acoustic model's [B, T, n_mels]
    (``"btc"``, models/acoustic_model.py:267-297), zero-padded past ``lengths[b]`` valid
    frames (the LengthRegulator's padding, models/variance_adaptor.py:223-264) — is
    either passed on every rank, or only on rank ``src`` (then broadcast once; the other
    ranks pass ``mel=None``).

    The utterances are split over the ranks by :func:`balance_by_length` (equal
    frame counts, not item counts); each rank runs ITS utterances as one ragged
    forward of ``gen`` (HiFiGANGenerator on this rank's GPU, ``hfg_forward_ex``) —
    no collective inside the forward — and the wavs are collected on rank ``dst`` by
    one ``dist.gather`` of equal-size (zero-padded) buffers.  Each wav equals the Generator run on that utterance alone (the
    ragged forward's per-utterance zero padding), so the result does not depend on
    the world size.

    Returns on rank ``dst``: the list of B wavs ``[output_length(lengths[b])]`` in
    batch order; on the other ranks None.  With ``dst=None`` no gather happens and
    every rank returns ``(indices, wavs)`` of its own utterances.
    """
    if not dist.is_initialized():
        raise RuntimeError("vocode_sharded needs an initialised torch.distributed process group")
    if mel_layout not in ("bct", "btc"):
        raise ValueError("mel_layout must be 'bct' or 'btc'")
    world, me = dist.get_world_size(group), dist.get_rank(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    if src is not None:
        mel, lengths = _broadcast_batch(mel, lengths, src, device, group)
    if mel is None or mel.dim() != 3:
        raise RuntimeError("vocode_sharded: expected a 3-D mel batch on every rank (or src=)")
    B = mel.shape[0]
    T = mel.shape[2] if mel_layout == "bct" else mel.shape[1]
    lens = [T] * B if lengths is None else [int(x) for x in lengths]
    if len(lens) != B or any(not 0 < n <= T for n in lens):
        raise ValueError(f"lengths must be {B} values in [1, {T}]")
    mine = balance_by_length(lens, world)[me]
    wavs: List[torch.Tensor] = []
    if mine:
        # this rank's utterances, trimmed to their own longest length
        t_max = max(lens[i] for i in mine)
        idx = torch.tensor(mine, dtype=torch.long)
        part = mel.index_select(0, idx.to(mel.device))
        part = part[:, :, :t_max] if mel_layout == "bct" else part[:, :t_max, :]
        part = part.to(device=device, dtype=torch.float32).contiguous()
        my_lens = [lens[i] for i in mine]
        with torch.no_grad():
            # a shard of equal lengths runs the plain (non-ragged) forward
            wav = gen(part, lengths=None if min(my_lens) == t_max else my_lens,
                      mel_layout=mel_layout)
        wavs = [wav[n, 0, :gen.output_length(lens[i])] for n, i in enumerate(mine)]
    if dst is None:
        return mine, wavs

    # gather: every rank knows every rank's items and wav lengths, so all ranks pad their
    # concatenated wavs to the largest rank's total and ONE dist.gather collects them on dst
    # (RCCL: one grouped call, no size exchange, no per-pair communicators)
    cdev = _coll_device(device, group)
    parts = balance_by_length(lens, world)
    sizes = [[gen.output_length(lens[i]) for i in parts[r]] for r in range(world)]
    pad = max(sum(s) for s in sizes)
    flat = torch.zeros(pad, dtype=torch.float32, device=cdev)
    if mine:
        flat[:sum(sizes[me])].copy_(torch.cat(wavs))
    gdst = dst if group is None else dist.get_global_rank(group, dst)
    bufs = ([torch.empty(pad, dtype=torch.float32, device=cdev) for _ in range(world)]
            if me == dst else None)
    dist.gather(flat, bufs, dst=gdst, group=group)
    if me != dst:
        return None
    out: List[Optional[torch.Tensor]] = [None] * B
    for n, i in enumerate(mine):
        out[i] = wavs[n]
    for r in range(world):
        if r == dst or not parts[r]:
            continue
        buf = bufs[r].to(device)
        off = 0
        for i, s in zip(parts[r], sizes[r]):
            out[i] = buf[off:off + s]
            off += s
    return out

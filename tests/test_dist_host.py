"""Multi-rank path on CPU with gloo (world_size 2): the one weight broadcast and
the utterance sharding used by bench.py.  On MI355X the same code runs on RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, root, q):
    import sys
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import __graft_entry__ as ge
        import importlib
        ge.load_package()
        hd = importlib.import_module(ge.PKG_NAME + ".dist")
        from oracle import config as C
        cfg = C.V2STAR
        spec = [(k, s) for k, s, _ in C.param_specs(cfg)]
        sd = None
        if rank == 0:
            sd = {k: torch.from_numpy(v) for k, v in C.make_state_dict(cfg, seed=9).items()}
        got = hd.broadcast_state_dict(sd, spec, torch.device("cpu"), src=0)
        ref = C.make_state_dict(cfg, seed=9)
        ok = all(np.array_equal(got[k].numpy(), ref[k]) for k in ref)
        # every utterance is owned by exactly one rank
        start, stop = hd.shard_range(13, world, rank)
        owned = torch.zeros(13)
        owned[start:stop] = 1
        dist.all_reduce(owned)
        q.put((rank, ok, bool(torch.all(owned == 1))))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_and_shard():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in procs)
    assert res == [(0, True, True), (1, True, True)]


def test_shard_range_and_balance(pkg):
    import importlib
    hd = importlib.import_module("tts_sambert_hifigan_amd.dist")
    for total in (1, 7, 64):
        for world in (1, 2, 3, 8):
            ranges = [hd.shard_range(total, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    lens = [63, 60, 61, 62, 63, 60, 10, 100]
    parts = hd.balance_by_length(lens, 3)
    assert sorted(i for p in parts for i in p) == list(range(len(lens)))
    loads = [sum(lens[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(lens)
    with pytest.raises(ValueError):
        hd.shard_range(4, 2, 2)


class _FakeGen:
    """CPU stand-in for HiFiGANGenerator with the same call surface vocode_sharded uses:
    a per-utterance function of the mel (hop 4) that zero-pads past each length, so a
    wav depends only on its own utterance's valid frames."""
    hop = 4

    def output_length(self, t):
        return self.hop * int(t)

    def __call__(self, mel, lengths=None, mel_layout="bct"):
        x = (mel if mel_layout == "bct" else mel.transpose(1, 2)).contiguous()
        B, C, T = x.shape
        lens = [T] * B if lengths is None else list(lengths)
        w = torch.arange(1, C + 1, dtype=torch.float32)
        out = torch.zeros(B, 1, self.hop * T)
        for b in range(B):
            v = (x[b, :, :lens[b]] * w[:, None]).sum(0).tanh()
            out[b, 0, :self.hop * lens[b]] = v.repeat_interleave(self.hop)
        return out


def _vs_worker(rank, world, port, root, q):
    import sys
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import __graft_entry__ as ge
        import importlib
        ge.load_package()
        hd = importlib.import_module(ge.PKG_NAME + ".dist")
        gen = _FakeGen()

        def _no_p2p(*a, **k):
            raise AssertionError("vocode_sharded must gather with one collective, not send/recv")

        dist.send = dist.recv = _no_p2p  # this process only
        g = torch.Generator().manual_seed(5)
        lens = [int(v) for v in torch.randint(3, 20, (11,), generator=g)]
        mel = torch.randn(11, 6, max(lens), generator=g)
        for b, n in enumerate(lens):
            mel[b, :, n:] = 0
        solo = [gen(mel[b:b + 1, :, :lens[b]])[0, 0] for b in range(11)]
        cpu = torch.device("cpu")
        ok = []
        # every rank passes the batch
        out = hd.vocode_sharded(gen, mel, lens, device=cpu)
        ok.append(out is None if rank != 0 else
                  all(torch.equal(a, b) for a, b in zip(out, solo)))
        # only rank 1 holds it ([B, T, C] layout); gather on rank 1
        out = hd.vocode_sharded(gen, mel.transpose(1, 2).contiguous() if rank == 1 else None,
                                lens if rank == 1 else None, mel_layout="btc", src=1, dst=1,
                                device=cpu)
        ok.append(out is None if rank != 1 else
                  all(torch.equal(a, b) for a, b in zip(out, solo)))
        # no gather: each rank's own share, the shares partition the batch
        mine, wavs = hd.vocode_sharded(gen, mel, lens, dst=None, device=cpu)
        ok.append(all(torch.equal(w, solo[i]) for i, w in zip(mine, wavs)))
        owned = torch.zeros(11)
        owned[mine] = 1
        dist.all_reduce(owned)
        ok.append(bool(torch.all(owned == 1)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_vocode_sharded_gather(world):
    """dist.vocode_sharded: length-balanced shards, per-rank forward, ONE dist.gather of
    zero-padded equal-size buffers (point-to-point send/recv are patched to fail); every gathered wav equals the utterance run alone (bitwise), with the batch
    given on every rank or broadcast from one, in both mel layouts."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_vs_worker, args=(r, world, port, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert res == [(r, [True] * 4) for r in range(world)]

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

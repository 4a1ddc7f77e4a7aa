"""World-size-N rehearsal of the sharded vocoding API on ONE GPU (every rank on cuda:0,
gloo backend): run as

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/tools/dist_world2_check.py

Rank 0 generates the weights and broadcasts them (dist.broadcast_state_dict); every rank
vocodes its length-balanced share through dist.vocode_sharded and the wavs are gathered on
rank 0, which compares them BITWISE with a single-process forward of the whole batch:
C3 (V1 [64, 80, 1024]) and C5 (the reference SAM-BERT acoustic model's 32 ragged
utterances, tests/golden/c5_sambert_b32.npz, also within 1e-4 of the reference wavs).
Rank 0 prints one JSON line.  Used by tests/test_gpu_dist.py.

HFG_DIST_BACKEND=nccl runs the same checks over RCCL (one rank per GPU: world size 1 on the
one-GPU box): ``dist.init_process_group("nccl", device_id=...)``, the weight broadcast and the
batch broadcast of ``vocode_sharded(..., src=0)`` on device buffers — the production path of
``bench.py --gpus N`` and of an 8-GPU node, short of an RCCL gather between two GPUs.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import importlib
    import __graft_entry__ as ge
    pkg = ge.load_package()
    pkg.load_library()
    hd = importlib.import_module(ge.PKG_NAME + ".dist")
    from oracle import config as C  # the checker's weights and fixtures

    backend = os.environ.get("HFG_DIST_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    # collective buffers: device memory for RCCL, host memory for gloo
    cdev = dev if backend == "nccl" else torch.device("cpu")
    res = {"world": world, "backend": dist.get_backend(), "checks": {}}
    gd = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gd, "golden_c5.json")))
    arr = np.load(os.path.join(gd, "c5_sambert_b32.npz"))
    for precision in ("f16x3", "fp32"):
        cfg = C.V1
        spec = [(k, s) for k, s, _ in C.param_specs(cfg)]
        sd0 = ({k: torch.from_numpy(v) for k, v in
                C.make_state_dict(cfg, seed=meta["vocoder_seed"]).items()} if rank == 0 else None)
        sd = hd.broadcast_state_dict(sd0, spec, cdev, src=0)
        res["weights_on"] = str(next(iter(sd.values())).device)
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
        gen.load_state_dict(sd)
        gen = gen.to(dev)
        cases = {}
        if precision == "f16x3":
            g = torch.Generator().manual_seed(1234)
            cases["C3_v1_64x80x1024"] = (torch.randn(64, 80, 1024, generator=g), None, "bct")
        mel_pred = torch.from_numpy(arr["mel_pred"])
        cases["C5_sambert_b32"] = (mel_pred, [int(x) for x in arr["lengths"]], "btc")
        for name, (mel, lens, layout) in cases.items():
            # the batch lives on rank 0 only: broadcast inside vocode_sharded (src=0)
            out = hd.vocode_sharded(gen, mel if rank == 0 else None, lens if rank == 0 else None,
                                    mel_layout=layout, src=0, dst=0, device=dev)
            torch.cuda.synchronize(dev)
            if rank != 0:
                continue
            with torch.no_grad():
                full = gen(mel.to(dev), lengths=lens, mel_layout=layout)
            torch.cuda.synchronize(dev)
            B = mel.shape[0]
            T = mel.shape[2] if layout == "bct" else mel.shape[1]
            L = [T] * B if lens is None else lens
            bitwise = all(torch.equal(out[b], full[b, 0, :gen.output_length(L[b])])
                          for b in range(B))
            chk = {"bitwise_vs_single_process": bitwise, "items": B,
                   "per_rank_items": [len(p) for p in hd.balance_by_length(L, world)]}
            if name.startswith("C5"):
                errs = [float(np.abs(out[b].cpu().numpy() - arr[f"wav_{b}"]).max())
                        for b in meta["full_wav"]]
                chk["max_err_vs_reference_wav"] = max(errs)
            res["checks"][f"{name}/{precision}"] = chk
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""One BASELINE leg at a time, for rocprofv3 (`rocprofv3 --kernel-trace --stats -d DIR --
python profiles/r03/legs.py LEG`): c1 (V1 [1,80,256]), c4 (V2* [16,80,2048]), c5 (32 ragged
utterances through the glue), mel (log-mel of 8 x 262144 samples), stream16 (16 streams, one
batched 64-frame chunk step).  Random weights (synth.py), 3 warm-up + 10 timed repetitions,
module defaults (bf16x3 via precision=)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(leg):
    import importlib
    import __graft_entry__ as ge
    pkg = ge.load_package()
    S = importlib.import_module(ge.PKG_NAME + ".synth")
    glue = importlib.import_module(ge.PKG_NAME + ".glue")
    mel = importlib.import_module(ge.PKG_NAME + ".mel")
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(1)

    def make(cfg):
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision="bf16x3").eval()
        gen.load_state_dict({k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg).items()})
        return gen.to(dev)

    if leg == "c1":
        gen, x = make(S.V1), torch.randn(1, 80, 256, generator=g).to(dev)
        fn = lambda: gen(x)  # noqa: E731
    elif leg == "c4":
        gen, x = make(S.V2STAR), torch.randn(16, 80, 2048, generator=g).to(dev)
        fn = lambda: gen(x)  # noqa: E731
    elif leg == "c5":
        gen = make(S.V1)
        lens = [int(v) for v in torch.randint(60, 64, (32,), generator=g)]
        x = torch.randn(32, max(lens), 80, generator=g).to(dev)
        fn = lambda: glue.vocode_acoustic(gen, x, lens)  # noqa: E731
    elif leg == "mel":
        ext, x = mel.MelSpectrogram(device=dev), torch.randn(8, 262144, generator=g).clamp(-1, 1).to(dev)
        fn = lambda: ext(x)  # noqa: E731
    elif leg == "stream16":
        gen = make(S.V1)
        sv = glue.StreamingVocoder(gen, chunk_frames=64, n_streams=16)
        feed = torch.randn(16, 80, 64, generator=g).to(dev)
        for s in range(16):
            sv.feed(feed[s, :, :sv.ctx], s)

        def fn():
            for s in range(16):
                sv.feed(feed[s], s)
            return sv.step()
    else:
        raise SystemExit(f"unknown leg {leg}")
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    print(f"{leg}: {1e3 * (time.perf_counter() - t0) / 10:.3f} ms per call")


if __name__ == "__main__":
    main(sys.argv[1])

"""Benchmark of the MI355X HiFi-GAN Generator hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--preset v1] [--batch 8] [--frames 1024]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N > 1` without a launcher environment starts the N ranks itself (torch.distributed.run
as a child process, before this process touches the GPU); under an external launcher the
WORLD_SIZE must equal N, or bench.py refuses to run (no mislabelled n_gpus).

A step = one Generator forward of a [batch, 80, frames] synthetic mel per GPU
(default batch 8 × 1024 frames = BASELINE config 2; 8 GPUs × 8 = config 3),
mel and weights resident in HBM before the timed region.  Utterances are
sharded over ranks (weak scaling); weights are generated on rank 0 and
broadcast once with RCCL.  Rank 0 prints ONE JSON line.

Timing: `value` is K uninstrumented steps of the production schedule (batch halves on
two HIP streams).  Roofline: a second timed pass of the same K steps on one stream with
every kernel launch bracketed by HIP events on that stream (libhifigan_hip profiling
mode); the dominant kernel's achieved TFLOP/s = its algorithmic FLOP ÷ its summed
launch time (with two streams the halves' intervals overlap, so they cannot be
attributed to one kernel).
Also: per-step HIP-event median (median of the timed steps), an
end-to-end figure with the H2D mel and D2H wav copies on the same stream, and (N=1)
`traffic` from two live rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of this same
workload, run as child processes before this process touches the GPU.
cpu_baseline: the oracle's PyTorch-CPU restatement (same ATen ops as the
reference) on this host's cores, rank 0 / N=1 only, on a bounded sample.

`value` is the whole-job aggregate (all ranks' samples ÷ the max-over-ranks time), as
the bench contract prescribes; the per-GPU figure the metric name speaks of is
`value_per_gpu` (identical at N=1).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402

METRIC = ("audio samples/sec/GPU (HiFi-GAN 80-mel→22.05 kHz) at 1/2/4/8 MI355X; RTF")
SAMPLE_RATE = 22050
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA dense (no sparsity)


# position of the NP (MFMA products per multiply-add) and FMT (split format) template
# arguments of the split-precision kernels, as hfg_profile_summary / rocprofv3 print them
_SPLIT_ARGS = {"conv1d_bf16x3": (8, 10), "ups_bf16x3": (4, 5), "resblock_bf16x3": (4, 5),
               "mrf_thin_mfma": (1, 2)}


def kernel_split(name: str):
    """(MFMA products per algorithmic multiply-add, split format "f16" / "bf16") of a
    split-precision kernel; (0, None) for the fp32-MFMA / VALU kernels."""
    base = name.split("<")[0].split("(")[0].strip()
    if base not in _SPLIT_ARGS or "<" not in name:
        return 0, None
    args = [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")]
    i_np, i_fmt = _SPLIT_ARGS[base]
    np_ = int(args[i_np]) if len(args) > i_np else 3
    fmt = "f16" if len(args) > i_fmt and args[i_fmt] == "1" else "bf16"
    return np_, fmt


def kernel_products(name: str) -> int:
    """MFMA products per algorithmic multiply-add of a kernel (0: fp32 MFMA / VALU): 3 for
    the split kernels (hi*hi + hi*lo + lo*hi, f16 or bf16 halves), 2 for the bf16w instances
    (NP = 2: lo(w) = 0 skipped)."""
    return kernel_split(name)[0]


def kernel_peak(name: str):
    """(peak in algorithmic fp32-conv TFLOP/s, description) for one kernel."""
    np_, fmt = kernel_split(name)
    if np_:
        return (PEAK_BF16_TFLOPS / np_,
                f"{fmt} dense MFMA 2.5 PFLOP/s / {np_} split products")
    return PEAK_FP32_TFLOPS, "fp32 MFMA 157.3 TFLOP/s"


def sustained_peak(pkg, dev_index, kind, cache={}):
    """Live dense TFLOP/s and shader clock of a pure MFMA stream on this GPU
    (hfg_probe_mfma_rate, csrc/probe.hip): kind 0 bf16 32x32x16, 1 fp32 32x32x2.
    ~0.1 s of full-chip MFMA load after the timed region."""
    if kind not in cache:
        import ctypes
        lib = pkg.load_library()
        tf, mhz = ctypes.c_double(0.0), ctypes.c_double(0.0)
        iters = 60000 if kind == 0 else 50000
        rc = lib.hfg_probe_mfma_rate(int(dev_index), int(kind), iters, ctypes.byref(tf),
                                     ctypes.byref(mhz))
        cache[kind] = (tf.value, mhz.value) if rc == 0 else None
    return cache[kind]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", default="v1", choices=["v1", "v2star"])
    ap.add_argument("--batch", type=int, default=8, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--precision", default="f16x3", choices=["fp32", "f16x3", "bf16x3", "bf16w"],
                    help="conv arithmetic: f16x3 split-precision MFMA (default: scaled f16 "
                         "halves, fp32-class products, every golden fixture within the exact-fp32 "
                         "bars, tests/test_gpu_stages.py), bf16x3 (bf16 halves: faster, ~16-bit "
                         "products), exact fp32 MFMA, or bf16w (weights stored as bf16: a "
                         "different model, parity against the bf16-rounded weights)")
    ap.add_argument("--also", nargs="*", default=["bf16x3", "fp32", "bf16w"],
                    help="extra precisions measured in the same run (reported under 'alt')")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group (and broadcast the weights) even at N = 1: "
                         "exercises the RCCL branch on a one-GPU box")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the other BASELINE configs (C1 latency + hipGraph, C4 V2*, C5 ragged)")
    ap.add_argument("--cpu-budget-s", type=float, default=30.0)
    ap.add_argument("--streams", type=int, default=2, choices=[1, 2],
                    help="HIP streams per forward (hfg_set_streams): 2 = batch halves overlap "
                         "(production default); per-kernel roofline figures always come from "
                         "a 1-stream profiled pass")
    ap.add_argument("--graph", action="store_true",
                    help="time the value pass as replays of one captured hipGraph of the forward "
                         "(both streams: fork / join events are captured); the per-kernel pass "
                         "stays eager")
    ap.add_argument("--no-profile", action="store_true",
                    help="do not bracket launches with HIP events (no roofline)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 FETCH_SIZE / WRITE_SIZE passes (traffic=null)")
    ap.add_argument("--sched", nargs="*", default=[], metavar="KNOB=V",
                    help="schedule overrides for A/B runs (hfg_debug_schedule_set, e.g. "
                         "RB_PERSIST=0); recorded in the line's config")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


# FETCH_SIZE / WRITE_SIZE corrections measured by profiles/pmc_calib.hip on gfx950
# (known 1 GiB streams; profiles/r02/pmc_calib.json): counter bytes / true bytes.
PMC_FETCH_SCALE = 0.5   # 4-B and 16-B per lane loads alike
PMC_WRITE_SCALE = 1.0   # 4-B and 16-B per lane stores alike


def _norm(name: str) -> str:
    name = name.split("(")[0]
    for pre in ("void ", "hfg::"):
        if name.startswith(pre):
            name = name[len(pre):]
    return name.replace(" ", "")


def _pmc_key(label: str, pmc: dict):
    """The rocprofv3 name (normalised) of a library profile label, or None: the whole-ResBlock
    labels name the persistent grid 'persist' and leave the non-persistent flag out, where the
    kernel's own name carries its last template argument (true / false)."""
    n = _norm(label)
    cands = [n, n + "_kernel"]
    if n.startswith("resblock_bf16x3<") and n.endswith(">"):
        args_ = n[len("resblock_bf16x3<"):-1].split(",")
        if args_[-1] == "persist":
            args_[-1] = "true"
        elif len(args_) == 6:
            args_.append("false")
        cands.append("resblock_bf16x3<" + ",".join(args_) + ">")
    return next((c for c in cands if c in pmc), None)


def _host_cores():
    """(threads to use, description): the CPUs this process may run on, capped by the
    cgroup CPU quota when one is set (a GPU box shows every host CPU in
    sched_getaffinity but grants a share of them)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:  # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except Exception:
            quota = None
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    use = min(aff, quota) if quota else aff
    env = os.environ.get("OMP_NUM_THREADS")
    desc = (f"{use} threads = sched_getaffinity {aff} CPUs"
            + (f" capped by the cgroup CPU quota {quota}" if quota else " (no cgroup quota)")
            + (f"; OMP_NUM_THREADS={env}" if env else "") + (f"; {model}" if model else ""))
    return use, desc


def pmc_traffic(argv_extra):
    """Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE and
    WRITE_SIZE in separate runs, no trace domains: MI355X_MICROARCH.md §HBM) of this
    workload on one stream.  Runs child processes; call before this process uses the GPU.
    Returns ({kernel: {fetch, write, bytes}}, note) or (None, reason)."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="hfg_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    per = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", counter, "-d", d, "-o", "run",
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__),
                   "--pmc-child", "--steps", "2", "--warmup", "1", "--streams", "1",
                   "--no-profile", "--no-extra", "--no-cpu-baseline", "--no-pmc"] + argv_extra + ["--also"]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, text=True)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} pass failed (rc {r.returncode}): " \
                             f"{r.stderr.strip().splitlines()[-1:] }"
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            vals = {}
            for fpath in files:
                with open(fpath) as f:
                    for row in csv.DictReader(f):
                        if row.get("Counter_Name") == counter:
                            vals.setdefault(_norm(row["Kernel_Name"]), []).append(
                                float(row["Counter_Value"]) * 1024.0)
            if not vals:
                return None, f"no {counter} rows in the rocprofv3 output"
            scale = PMC_FETCH_SCALE if counter == "FETCH_SIZE" else PMC_WRITE_SCALE
            for k, v in vals.items():
                per.setdefault(k, {})["fetch" if counter == "FETCH_SIZE" else "write"] = \
                    sum(v) / len(v) / scale
        for v in per.values():
            v["bytes"] = v.get("fetch", 0.0) + v.get("write", 0.0)
        return per, ("live rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes of this workload "
                     f"(1 stream, 3 forwards); FETCH_SIZE / {PMC_FETCH_SCALE}, WRITE_SIZE / "
                     f"{PMC_WRITE_SCALE} (profiles/pmc_calib.hip calibration), KiB x 1024")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cpu_baseline(cfg, sd, batch, frames, budget_s):
    """Oracle (PyTorch-CPU restatement) on host cores, on the bench line's own workload:
    [batch, 80, frames] (C2 = [8, 80, 1024]), best of N runs after a warm-up, as many as fit
    in ~budget_s (at least one).  The one-utterance [1, 80, frames] rate (the
    CPU runs batch 8 at about half its batch-1 rate) is reported beside it as `batch1`."""
    from oracle import config as OC, hifigan_torch, prng  # the CPU baseline leg only
    cfg = OC.GenConfig(**cfg.kwargs())
    threads, cores_desc = _host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    tsd = hifigan_torch.to_torch_state(sd)
    mel = torch.from_numpy(prng.mel_input(1234, (batch, cfg.n_mels, frames)))

    def best_of(x, budget):
        best, runs, t_all = None, 0, time.perf_counter()
        while runs < 1 or (time.perf_counter() - t_all + (best or 0.0) < budget and runs < 3):
            t0 = time.perf_counter()
            with torch.no_grad():
                wav = hifigan_torch.generator_forward(tsd, cfg, x)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
            runs += 1
        return best, runs, wav.numel()

    with torch.no_grad():
        hifigan_torch.generator_forward(tsd, cfg, mel[:1, :, :32])  # warm-up
    best, runs, samples = best_of(mel, budget_s)
    best1, runs1, samples1 = best_of(mel[:1], min(budget_s, 8.0))
    torch.set_num_threads(prev)
    return {"value": samples / best, "unit": "audio samples/s", "cores": threads,
            "kind": "port",
            "sample": f"the bench workload itself: [{batch},{cfg.n_mels},{frames}] -> "
                      f"{samples} samples, best of {runs} after warm-up, oracle/hifigan_torch.py "
                      "(same ATen ops as the reference, SURVEY.md §8(d))",
            "cores_note": cores_desc,
            "rtf": best / (samples / SAMPLE_RATE),
            "batch1": {"value": samples1 / best1, "runs": runs1,
                       "sample": f"one utterance [1,{cfg.n_mels},{frames}], best of {runs1}"}}


def extra_configs(pkg, S, dev, precision, steps=5):
    """The other BASELINE.json configs, measured on this GPU (rank 0, N=1):
    C1 V1 [1,80,256] latency, eager vs a captured hipGraph replay (torch.cuda.graph
    around the same forward: 78 launches on the capture stream); C4 pinned V2*
    [16,80,2048]; C5 the acoustic->vocoder glue on 32 ragged utterances of 60-63
    frames in the acoustic model's [B,T,80] layout."""
    import importlib
    glue = importlib.import_module(ge.PKG_NAME + ".glue")
    out = {}

    def timed(fn, n):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / n

    def make(cfg):
        # module defaults (verify_weights off: no per-forward host sync, hifigan.py)
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
        gen.load_state_dict({k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg).items()})
        return gen.to(dev)

    def module_vs_abi(gen, mel, n):
        """gen(mel) as a reference user calls it vs the raw C ABI on preallocated buffers
        (same handle, same streams): per-forward wall time of n back-to-back forwards, and
        the host time of one call (the module's Python wrapper + the ABI's launches)."""
        h = gen.hip_handle(dev)
        B, _, T = mel.shape
        out_len = h.out_len(T)
        wav = torch.empty((B, 1, out_len), device=dev)
        ws_b = h.workspace_bytes(B, T)
        ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream

        def raw():
            h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_b, st)

        def mod():
            gen(mel)

        res = {}
        for name, fn in (("abi", raw), ("module", mod)):
            for _ in range(3):
                fn()
            res[name + "_ms"] = timed(fn, n) * 1e3
            torch.cuda.synchronize(dev)
            host = []
            for _ in range(5):
                t0 = time.perf_counter()
                fn()
                host.append(time.perf_counter() - t0)
                torch.cuda.synchronize(dev)
            res[name + "_host_us_per_call"] = sorted(host)[2] * 1e6
        gen.verify_weights = True
        for _ in range(2):
            mod()
        res["module_verify_weights_ms"] = timed(mod, n) * 1e3
        gen.verify_weights = False
        res["overhead_pct"] = 100.0 * (res["module_ms"] / res["abi_ms"] - 1.0)
        res["overhead_us"] = 1e3 * (res["module_ms"] - res["abi_ms"])
        res["note"] = ("gen(mel) through the drop-in module (defaults: no per-forward weight "
                       "hash) vs hfg_forward_ws on preallocated buffers, n back-to-back forwards; "
                       "host_us_per_call = wall time of one call (launches are asynchronous); "
                       "module_verify_weights_ms = the opt-in content hash (a stream sync per "
                       "forward)")
        return res

    g = torch.Generator().manual_seed(1234)
    with torch.no_grad():
        gen = make(S.V1)
        mel = torch.randn(1, 80, 256, generator=g).to(dev)
        for _ in range(3):
            gen(mel)
        eager = timed(lambda: gen(mel), 20)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                gen(mel)
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            wav_g = gen(mel)
        graph.replay()
        replay = timed(graph.replay, 20)
        ok = bool(torch.equal(wav_g, gen(mel)))
        out["C1_v1_1x80x256"] = {"eager_ms": eager * 1e3, "hipgraph_ms": replay * 1e3,
                                 "samples_per_s_hipgraph": 65536 / replay,
                                 "rtf_hipgraph": replay / (65536 / SAMPLE_RATE),
                                 "graph_equals_eager": ok}
        # one StreamingVocoder chunk (glue.py): 64 new frames + the receptive-field context
        # (15 frames for V1) on each side, one utterance
        ctx = gen.receptive_field_frames()
        chunk = torch.randn(1, 80, 64 + 2 * ctx, generator=g).to(dev)
        for _ in range(3):
            gen(chunk)
        t_chunk = timed(lambda: gen(chunk), 20)
        out["streaming_chunk_v1_64f"] = {"frames_in": 64 + 2 * ctx, "frames_emitted": 64,
                                         "ms": t_chunk * 1e3,
                                         "rtf": t_chunk / (64 * 256 / SAMPLE_RATE)}
        out["module_forward_C1_1x80x256"] = module_vs_abi(gen, mel, 50)
        # many concurrent streams batched into one forward per step (glue.StreamingVocoder
        # with n_streams): steady state, every stream contributes one 64-frame chunk a step
        for n_streams in (16, 64):
            sv = glue.StreamingVocoder(gen, chunk_frames=64, n_streams=n_streams)
            feed = torch.randn(n_streams, 80, 64, generator=g).to(dev)
            for s_ in range(n_streams):
                sv.feed(feed[s_, :, :ctx], s_)

            def one_step():
                for s_ in range(n_streams):
                    sv.feed(feed[s_], s_)
                return sv.step()

            for _ in range(3):
                one_step()
            t_step = timed(one_step, 20)
            out[f"streaming_{n_streams}_streams_v1_64f"] = {
                "ms_per_step": t_step * 1e3, "streams": n_streams,
                "chunk_latency_ms": t_step * 1e3,
                "audio_s_per_wall_s": n_streams * 64 * 256 / SAMPLE_RATE / t_step,
                "rtf_per_stream": t_step / (64 * 256 / SAMPLE_RATE),
                "note": "glue.StreamingVocoder(n_streams): feed 64 frames to every stream, one "
                        "step() = one batched forward of all chunks (64 + 2 x context frames "
                        "each), bounded per-stream buffers; wall time incl. host work"}
        del gen
        gen = make(S.V2STAR)
        mel = torch.randn(16, 80, 2048, generator=g).to(dev)
        for _ in range(2):
            gen(mel)
        t = timed(lambda: gen(mel), steps)
        out["C4_v2star_16x80x2048"] = {"ms_per_step": t * 1e3, "samples_per_s": 16 * 2048 * 256 / t,
                                       "rtf": t / (16 * 2048 * 256 / SAMPLE_RATE)}
        del gen
        gen = make(S.V1)
        mel8 = torch.randn(8, 80, 1024, generator=g).to(dev)
        out["module_forward_C2_8x80x1024"] = module_vs_abi(gen, mel8, steps)
        del mel8
        lens = [int(x) for x in torch.randint(60, 64, (32,), generator=g)]
        mel_pred = torch.randn(32, max(lens), 80, generator=g).to(dev)
        for _ in range(2):
            glue.vocode_acoustic(gen, mel_pred, lens)
        t = timed(lambda: glue.vocode_acoustic(gen, mel_pred, lens), steps)
        valid = sum(lens) * 256
        out["C5_glue_32_ragged_60to63"] = {"ms_per_step": t * 1e3, "samples_per_s": valid / t,
                                           "frames": lens[:8] + ["..."],
                                           "note": "vocoder half of config 5; the SAM-BERT "
                                                   "acoustic model is CPU reference code (out of scope)"}
        # the mel row: log-mel of the C2 workload's audio, and the
        # 16 kHz -> 22.05 kHz resampler on 8 one-second utterances
        melmod = importlib.import_module(ge.PKG_NAME + ".mel")
        ext = melmod.MelSpectrogram(device=dev)
        audio = torch.randn(8, 262144, generator=g).clamp(-1, 1).to(dev)
        for _ in range(2):
            ext(audio)
        t = timed(lambda: ext(audio), 20)
        out["mel_8x262144"] = {"ms": t * 1e3, "frames_per_s": 8 * (262144 // 256 + 1) / t,
                               "audio_samples_per_s": 8 * 262144 / t,
                               "note": "hfg_mel_forward: framing + real FFT (float64 Stockham in LDS) + mel + log in one launch"}
        rs = melmod.Resample(16000, 22050, device=dev)
        a16 = torch.randn(8, 16000, generator=g).clamp(-1, 1).to(dev)
        for _ in range(2):
            rs(a16)
        t = timed(lambda: rs(a16), 20)
        out["resample_16k_to_22k_8x1s"] = {"ms": t * 1e3, "out_samples_per_s": 8 * 22050 / t}
    return out


def self_launch(args) -> int:
    """`--gpus N > 1` without a launcher: start N rank processes of this same command
    through torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and
    return its exit code.  Called before this process makes any GPU call (the ranks are
    children; this process never initialises HIP)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HFG_BENCH_SELF_LAUNCHED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(self_launch(args))
    rank, world, local_rank = 0, 1, 0
    if "RANK" in os.environ:
        rank, world, local_rank = (int(os.environ["RANK"]), int(os.environ.get("WORLD_SIZE", "1")),
                                   int(os.environ.get("LOCAL_RANK", "0")))
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE {world} "
                         "ranks: refusing to report a mislabelled n_gpus")
    pmc, pmc_note = None, "not collected (--no-pmc or N > 1)"
    under_profiler = "rocprof" in os.environ.get("LD_PRELOAD", "")
    if world == 1 and not args.no_pmc and not args.pmc_child and not under_profiler:
        # before this process initialises the GPU: the passes are child processes
        print("[bench] PMC traffic passes", file=sys.stderr, flush=True)
        pmc, pmc_note = pmc_traffic(["--preset", args.preset, "--batch", str(args.batch),
                                     "--frames", str(args.frames), "--precision", args.precision]
                                    + (["--sched"] + args.sched if args.sched else []))
    assert torch.cuda.is_available(), "bench.py needs MI355X GPUs"
    dev_index = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    use_dist = world > 1 or args.force_dist
    if use_dist:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"[bench] process group has {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")

    pkg = ge.load_package()
    pkg.load_library()
    for kv in args.sched:  # before any handle exists (read at hfg_create)
        k, v = kv.split("=", 1)
        pkg.schedule_override(k, int(v))
    import importlib
    hdist = importlib.import_module(ge.PKG_NAME + ".dist")
    S = importlib.import_module(ge.PKG_NAME + ".synth")  # random-init weights of the config
    global PREC
    PREC = importlib.import_module(ge.PKG_NAME + ".precision")  # documented scale limits

    cfg = S.PRESETS[args.preset]
    spec = [(k, s) for k, s, _ in S.param_specs(cfg)]
    sd_np = S.random_state_dict(cfg, seed=0) if rank == 0 else None
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    if use_dist:
        sd = hdist.broadcast_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}
                                        if rank == 0 else None, spec, coll_dev, src=0)
    else:
        sd = {k: torch.from_numpy(v) for k, v in sd_np.items()}
    # this rank's utterances of the global batch (weak scaling: batch per GPU fixed)
    global_batch = args.batch * world
    start, stop = hdist.shard_range(global_batch, world, rank)
    B, T = stop - start, args.frames
    gmel = torch.Generator().manual_seed(1234)
    mel_all = torch.randn(global_batch, cfg.n_mels, T, generator=gmel)
    mel = mel_all[start:stop].contiguous().to(dev)
    stream = torch.cuda.current_stream(dev)
    host_sd = {k: v.detach().cpu() for k, v in sd.items()}

    def measure(precision):
        """Warm-up, then EXACTLY args.steps timed forwards bracketed by barrier +
        synchronize; returns (max-over-ranks seconds, per-kernel profile, out_len)."""
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
        gen.load_state_dict(host_sd)
        h = gen.hip_handle(dev)
        out_len = h.out_len(T)
        wav = torch.empty((B, 1, out_len), dtype=torch.float32, device=dev)
        h.set_streams(1)
        ws_bytes = h.workspace_bytes(B, T)
        h.set_streams(args.streams)
        ws_bytes = max(ws_bytes, h.workspace_bytes(B, T))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)

        def step():
            h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes,
                         stream.cuda_stream)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        eager_step = step
        if args.graph:
            # one forward captured on a side stream, replayed on `stream` (the handle forks its
            # second half onto its internal stream with events, which the capture records)
            side = torch.cuda.Stream(dev)
            side.wait_stream(stream)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                with torch.cuda.graph(graph, stream=side):
                    h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(),
                                 ws_bytes, side.cuda_stream)
            stream.wait_stream(side)
            torch.cuda.synchronize(dev)

            def step():
                with torch.cuda.stream(stream):
                    graph.replay()

            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize(dev)
        profile = not args.no_profile
        # with 2 streams the timed loop runs uninstrumented (its per-launch intervals would
        # overlap anyway), and graph replays bypass the library's launcher (no per-launch
        # events); the per-kernel events then come from the eager 1-stream pass below
        inline_prof = profile and args.streams == 1 and not args.graph
        if inline_prof:
            h.profile_reset()
            h.set_profiling(True)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        evs[0].record(stream)
        for i in range(args.steps):
            step()
            evs[i + 1].record(stream)   # the forward joins its aux stream back into `stream`
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
        ev_median[precision] = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else \
            0.5 * (step_ms[len(step_ms) // 2 - 1] + step_ms[len(step_ms) // 2])
        if use_dist:
            dist.barrier()
            t = torch.zeros(world, dtype=torch.float64, device=coll_dev)
            t[rank] = elapsed
            dist.all_reduce(t)  # every rank's time (the others contribute 0)
            rank_ms[precision] = [1000.0 * float(v) / args.steps for v in t.tolist()]
            elapsed = max(float(v) for v in t.tolist())
        else:
            rank_ms[precision] = [1000.0 * elapsed / args.steps]
        prof = {}
        if profile:
            if inline_prof:
                h.set_profiling(False)
                prof = h.profile_summary()
            else:
                # per-kernel times: with the batch halves overlapping, a dispatch's interval
                # also covers the other half's kernels, so the roofline pass times the same
                # K steps again on one stream, every launch bracketed by HIP events on it
                h.set_streams(1)
                for _ in range(args.warmup):
                    eager_step()
                torch.cuda.synchronize(dev)
                h.profile_reset()
                h.set_profiling(True)
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    eager_step()
                torch.cuda.synchronize(dev)
                prof_ms[precision] = 1000.0 * (time.perf_counter() - t1) / args.steps
                h.set_profiling(False)
                prof = h.profile_summary()
                h.set_streams(args.streams)
        # content hash of the value pass's output (hfg_checksum32): same-box A/B builds that must
        # be bitwise equal show it (profiles/r06/lib_ab.sh)
        wav_sum[precision] = int(pkg._lib.checksum32([wav])[0]) & 0xffffffff
        if precision == args.precision and not args.pmc_child:
            e2e[precision] = end_to_end(eager_step, wav)
        del ws, wav
        return elapsed, prof, out_len

    def end_to_end(step, wav_d):
        """K steps of: H2D of the mel from pinned host memory, the forward, D2H of the wav
        into pinned host memory, all on the launch stream (SURVEY.md §8(d) end-to-end)."""
        mel_h = mel.cpu().pin_memory()
        wav_h = torch.empty(wav_d.shape, dtype=torch.float32).pin_memory()
        mel_d = mel

        def one():
            mel_d.copy_(mel_h, non_blocking=True)
            step()
            wav_h.copy_(wav_d, non_blocking=True)

        one()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            one()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t1) / args.steps
        return {"ms_per_step": dt * 1e3, "samples_per_s": wav_d.numel() / dt,
                "note": "H2D mel (pinned) + forward + D2H wav (pinned) on one stream, K steps; "
                        "the copies are not overlapped with the next step's compute"}

    prof_ms = {}  # ms/step of the 1-stream roofline pass, per precision
    rank_ms = {}  # per-rank ms/step of the value pass, per precision
    ev_median = {}  # per-step HIP-event median (ms) of the value pass, per precision
    wav_sum = {}  # hfg_checksum32 of the value pass's wav, per precision
    e2e = {}
    def progress(msg):
        """one stderr line per phase (a long run then shows it is alive)"""
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    progress(f"measuring {args.precision}")
    elapsed, prof, out_len = measure(args.precision)
    alt = {}
    for prec in args.also:
        if prec != args.precision:
            progress(f"measuring {prec}")
            alt[prec] = measure(prec)

    samples_total = global_batch * out_len * args.steps
    value = samples_total / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    if rank != 0:
        if use_dist:
            dist.destroy_process_group()
        return

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "audio samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else args.precision,
        "dtype_note": PREC.dtype_note(args.precision),
        "precision_limit": ({f"x{k:g}": v for k, v in PREC.BF16X3_SCALE_LIMITS.items()}
                            if args.precision == "bf16x3" else None),
        "precision_measured": PREC.MEASURED.get(args.precision),
        "data": "synthetic: mel ~ N(0,1) (torch seed 1234), random default-init weights "
                "U(+-1/sqrt(fan_in)) of the preset (synth.py; no checkpoint ships)",
        "config": {
            "workload": f"HiFi-GAN {args.preset.upper()} Generator forward, mel [{args.batch},"
                        f"{cfg.n_mels},{T}] per GPU -> wav [{args.batch},1,{out_len}]",
            "batch_per_gpu": args.batch,
            "frames": T,
            "global_batch": global_batch,
            **({"schedule_overrides": dict(pkg.schedule_overrides())} if args.sched else {}),
            "parallelism": (f"dp{world} (utterance-sharded, "
                            f"{'RCCL' if args.dist_backend == 'nccl' else 'gloo'} weight broadcast at init)"
                            if use_dist else "dp1"),
        },
        "value_per_gpu": value / world,
        "per_rank_ms_per_step": rank_ms.get(args.precision),
        "world_size_observed": dist.get_world_size() if use_dist else 1,
        "dist_backend": args.dist_backend if use_dist else None,
        "launch": ("self-launched torch.distributed.run" if os.environ.get("HFG_BENCH_SELF_LAUNCHED")
                   else "external launcher" if "RANK" in os.environ else "single process"),
        "value_note": "value = whole-job aggregate (all ranks' samples / max-over-ranks time, the "
                      "bench contract); value_per_gpu = value / n_gpus",
        "value_pass": ("hipGraph replays of one captured forward" if args.graph
                       else "eager forwards (hfg_forward_ws per step)") +
                      f", {args.streams} stream(s)",
        "rtf": (elapsed / args.steps) / (args.batch * out_len / SAMPLE_RATE),
        "step_ms_hipevent_median": ev_median.get(args.precision),
        "wav_checksum32": f"{wav_sum[args.precision]:08x}" if args.precision in wav_sum else None,
        "samples_per_s_hipevent_median": (args.batch * out_len / (ev_median[args.precision] * 1e-3)
                                          if ev_median.get(args.precision) else None),
    }
    if args.precision in e2e:
        line["end_to_end"] = e2e[args.precision]
    def roofline(prof, ms_per_step):
        dom_name, dom = max(prof.items(), key=lambda kv: kv[1]["ms"])
        achieved = dom["flop"] / (dom["ms"] * 1e-3) / 1e12
        peak, peak_note = kernel_peak(dom_name)
        return {"bound": "mfma", "kernel": dom_name, "achieved": achieved, "peak": peak,
                "peak_note": peak_note, "unit": "TFLOP/s", "frac": achieved / peak,
                "avg_launch_ms": dom["ms"] / dom["launches"],
                "flop_per_launch": dom["flop"] / dom["launches"],
                "share_of_step": dom["ms"] / args.steps / ms_per_step}

    if alt:
        line["alt"] = {}
        for prec, (el, pr, ol) in alt.items():
            v = global_batch * ol * args.steps / el
            entry = {"value": v, "ms_per_step": 1000.0 * el / args.steps,
                     "wav_checksum32": f"{wav_sum[prec]:08x}" if prec in wav_sum else None,
                     "rtf": (el / args.steps) / (args.batch * ol / SAMPLE_RATE),
                     "speedup_vs_headline": v / value,
                     "parity": ("atol 1e-4 vs the oracle run on the bf16-rounded weights "
                                "(tests/test_gpu_bf16w.py)" if prec == "bf16w" else PREC.note(prec))}
            if pr:
                entry["roofline"] = roofline(pr, prof_ms.get(prec, 1000.0 * el / args.steps))
                entry["kernels"] = {k: {"launches": q["launches"] // args.steps,
                                        "ms_per_step": q["ms"] / args.steps}
                                    for k, q in sorted(pr.items(), key=lambda kv: -kv[1]["ms"])}
            line["alt"][prec] = entry
    if prof:
        tot_ms = sum(v["ms"] for v in prof.values()) / args.steps
        dom_name, dom = max(prof.items(), key=lambda kv: kv[1]["ms"])
        achieved = dom["flop"] / (dom["ms"] * 1e-3) / 1e12
        traffic = None
        if pmc and _norm(dom_name) in pmc:
            traffic = pmc[_norm(dom_name)]["bytes"]
        peak, peak_note = kernel_peak(dom_name)
        line["roofline"] = {
            "bound": "mfma",
            "kernel": dom_name,
            "achieved": achieved,
            "peak": peak,
            "peak_note": peak_note,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "traffic": traffic,
            "traffic_note": pmc_note,
            "traffic_over_alg_bytes": (traffic / (dom["bytes"] / dom["launches"])
                                       if traffic else None),
            "launches_per_step": dom["launches"] / args.steps,
            "avg_launch_ms": dom["ms"] / dom["launches"],
            "flop_per_launch": dom["flop"] / dom["launches"],
            "alg_bytes_per_launch": dom["bytes"] / dom["launches"],
            "share_of_step": dom["ms"] / args.steps / prof_ms.get(args.precision, ms_per_step),
        }
        n_prod = kernel_products(dom_name)
        sp = sustained_peak(pkg, dev_index, 0 if n_prod else 1)
        if sp:
            n_prod = max(n_prod, 1)
            alg_peak = sp[0] / n_prod
            line["roofline"]["peak_sustained"] = {
                "mfma_dense_TFLOPs": sp[0], "clock_MHz": sp[1],
                "algorithmic_TFLOPs": alg_peak, "frac": achieved / alg_peak,
                "note": "pure MFMA stream on random operands, 2 blocks x 4 waves per CU, "
                        "measured live after the timed region on this GPU (csrc/probe.hip, "
                        f"hfg_probe_mfma_rate); divided by {n_prod} product(s) per "
                        "multiply-add like 'peak'.  The DVFS ceiling a matrix kernel meets "
                        "under full-chip load; 'peak' stays the datasheet figure"}
        if args.precision in prof_ms:
            line["roofline"]["pass"] = (
                "per-kernel HIP-event times from a second timed pass of the same K steps on "
                f"1 stream ({prof_ms[args.precision]:.3f} ms/step); the value pass runs "
                f"{args.streams} streams uninstrumented (overlapping batch halves make "
                "per-kernel intervals overlap)")
        all_flop = sum(v["flop"] for v in prof.values()) / args.steps
        all_bytes = sum(v["bytes"] for v in prof.values()) / args.steps
        step_s = elapsed / args.steps
        issue = {"f16x3": 3.0, "bf16x3": 3.0, "bf16w": 2.0}.get(args.precision, 1.0)
        line["roofline_step"] = {
            "compute_TFLOPs": all_flop / step_s / 1e12,
            "mfma_issue_frac": (all_flop * issue / step_s / 1e12 /
                                (PEAK_BF16_TFLOPS if args.precision != "fp32" else PEAK_FP32_TFLOPS)),
            "mfma_issue_note": (f"algorithmic FLOP x {issue:.0f} f16/bf16 MFMA products per "
                                "multiply-add / step time / 2.5 PF dense peak" if args.precision != "fp32" else
                                "algorithmic FLOP / step time / 157.3 TF fp32 MFMA peak"),
            "hbm_model_GBs": all_bytes / step_s / 1e9,
            "hbm_model_frac": all_bytes / step_s / 1e9 / PEAK_HBM_GBS,
            "kernel_time_ms": tot_ms,
            "note": "algorithmic FLOP and the per-launch algorithmic bytes of the kernels as "
                    "launched (a whole-ResBlock launch counts only its own input, output and "
                    "weights) per step / step time",
        }
        # SURVEY.md §8(d) canonical layer-streaming byte model (fp32, every conv streams
        # its input and output, weights once per forward): the north-star HBM-roofline figure
        bpf = S.layer_streaming_bytes_per_frame(cfg)
        gpu_bytes = B * T * bpf + S.param_bytes(cfg)  # per GPU per step
        line["roofline_step"]["hbm_canonical"] = {
            "bytes_per_frame": bpf,
            "bytes_per_sample": gpu_bytes / (B * out_len),
            "GBs_per_gpu": gpu_bytes / step_s / 1e9,
            "frac": gpu_bytes / step_s / 1e9 / PEAK_HBM_GBS,
            "note": "equivalent bandwidth of the layer-streaming model at the measured step "
                    "time; the fused kernels move fewer bytes (PMC traffic in roofline)",
        }
        if pmc:
            # measured HBM bytes of one step: every kernel's PMC bytes per launch x its launches
            # per step (1-stream pass counts; the 2-stream value pass moves the same bytes)
            meas, missing = 0.0, []
            for k, v in prof.items():
                pk = _pmc_key(k, pmc)
                if pk:
                    meas += pmc[pk]["bytes"] * v["launches"] / args.steps
                else:
                    missing.append(k)
            line["roofline_step"]["hbm_pmc"] = {
                "bytes_per_step": meas, "GBs": meas / step_s / 1e9,
                "frac": meas / step_s / 1e9 / PEAK_HBM_GBS,
                "kernels_without_pmc": missing,
                "note": "measured: sum of per-kernel PMC bytes per step / value-pass step time"}
        line["kernels"] = {k: {"launches": v["launches"] // args.steps,
                               "ms_per_step": v["ms"] / args.steps,
                               "TFLOPs": v["flop"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else None,
                           "pmc_bytes_per_launch": (pmc[_pmc_key(k, pmc)]["bytes"]
                                                    if pmc and _pmc_key(k, pmc) else None),
                           "alg_bytes_per_launch": v["bytes"] / v["launches"]}
                           for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])}
    if world == 1 and not args.no_extra:
        line["extra_configs"] = extra_configs(pkg, S, dev, args.precision)
    if world == 1 and not args.no_cpu_baseline:
        cfg_np = S.random_state_dict(cfg, seed=0) if sd_np is None else sd_np
        progress("CPU baseline")
        line["cpu_baseline"] = cpu_baseline(cfg, cfg_np, B, T, args.cpu_budget_s)
        line["cpu_baseline"]["gpu_over_cpu"] = value / line["cpu_baseline"]["value"]
    print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

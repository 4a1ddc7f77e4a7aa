"""Build libhifigan_hip.so in-tree with hipcc for gfx950 (no torch, no JIT cache).

    python tts-sambert_hifigan_amd/build.py          # or __graft_entry__.build()
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_NAME = "libhifigan_hip.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
SOURCES = ["conv_kernels.hip", "conv_bf16x3.hip", "conv16_bf16x3.hip", "resblock_bf16x3.hip",
           "resblock16_bf16x3.hip", "mrf_thin.hip", "mrf_thin_mfma.hip",
           "conv_ws_bf16x3.hip", "probe.hip", "hifigan_capi.cpp", "mel_kernels.hip", "mel_capi.cpp"]
HEADERS = ["kernels.h", "mel_kernels.h", "epilogue.h", "bf16x3_common.h", os.path.join("..", "..", "include", "hifigan_hip.h"),
           os.path.join("..", "..", "include", "hifigan_hip_inspect.h")]

OBJ_DIR = os.path.join(PKG_DIR, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950",
    # code object v5: loadable by both /opt/rocm (7.2) and torch's bundled HIP runtime
    "-mcode-object-version=5",
    "-O3", "-std=c++17", "-fPIC",
    "-Wall", "-Wno-unused-result",
]


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def _obj(src: str) -> str:
    return os.path.join(OBJ_DIR, os.path.splitext(src)[0] + ".o")


def _compile(src: str, verbose: bool):
    cmd = [HIPCC, *FLAGS, "-c", os.path.join(CSRC, src), "-o", _obj(src) + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        return src, res.stdout + res.stderr
    os.replace(_obj(src) + ".tmp", _obj(src))
    return src, None


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile the HIP kernels + C ABI into ``libhifigan_hip.so`` next to this file: one
    object per source (in parallel, only the stale ones), then one link."""
    if not force and not _stale():
        return LIB_PATH
    os.makedirs(OBJ_DIR, exist_ok=True)
    hdr_t = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS
                if os.path.exists(os.path.join(CSRC, h)))
    todo = [src for src in SOURCES
            if force or not os.path.exists(_obj(src))
            or os.path.getmtime(_obj(src)) < max(hdr_t, os.path.getmtime(os.path.join(CSRC, src)))]
    jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(jobs) as ex:
        errs = [(src, err) for src, err in ex.map(lambda s_: _compile(s_, verbose), todo) if err]
    if errs:
        for src, err in errs:
            sys.stderr.write(f"--- {src}\n{err}")
        raise RuntimeError(f"hipcc failed on {', '.join(s_ for s_, _ in errs)}")
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC",
           *[_obj(src) for src in SOURCES], "-o", tmp]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"hipcc link failed with exit code {res.returncode}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))

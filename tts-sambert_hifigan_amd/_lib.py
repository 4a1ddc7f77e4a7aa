"""ctypes binding of libhifigan_hip.so (C ABI: include/hifigan_hip.h).

The library is the product path; there is no fallback.  Loading fails loudly
when the .so is missing (build it with ``__graft_entry__.build()`` or
``python tts-sambert_hifigan_amd/build.py``).

``torch`` is imported before the library is opened so that the library's
``libamdhip64.so.7`` dependency binds to the HIP runtime torch already loaded
(same SONAME) — one HIP runtime per process, and torch's streams and device
pointers are valid handles for the library.
"""
from __future__ import annotations

from typing import Optional

import ctypes
import os
from ctypes import (POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_size_t, c_void_p,
                    c_float)

import torch  # noqa: F401  (see module docstring: bind torch's HIP runtime first)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libhifigan_hip.so")

HFG_MAX_STAGES = 8
HFG_MAX_RES = 8
HFG_MAX_DIL = 8

ERRORS = {0: "OK", -22: "EINVAL", -12: "ENOMEM", -19: "ENODEV", -11: "EAGAIN", -5: "EIO"}


class HipExtensionMissing(RuntimeError):
    pass


class HfgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hifigan_hip error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class HfgForwardOpts(ctypes.Structure):
    _fields_ = [("mel_layout", c_int32), ("lengths", c_void_p)]


MEL_LAYOUTS = {"bct": 0, "btc": 1}


class HfgConfig(ctypes.Structure):
    _fields_ = [
        ("n_mels", c_int32),
        ("n_up", c_int32),
        ("up_rates", c_int32 * HFG_MAX_STAGES),
        ("up_kernels", c_int32 * HFG_MAX_STAGES),
        ("c0", c_int32),
        ("n_res", c_int32),
        ("res_kernels", c_int32 * HFG_MAX_RES),
        ("n_dil", c_int32 * HFG_MAX_RES),
        ("dil", (c_int32 * HFG_MAX_DIL) * HFG_MAX_RES),
        ("dtype", c_int32),
    ]


DTYPES = {"fp32": 0, "bf16x3": 1, "bf16w": 2, "f16x3": 3}


class HfgMrfConfig(ctypes.Structure):
    _fields_ = [
        ("channels", c_int32),
        ("n_res", c_int32),
        ("res_kernels", c_int32 * HFG_MAX_RES),
        ("n_dil", c_int32 * HFG_MAX_RES),
        ("dil", (c_int32 * HFG_MAX_DIL) * HFG_MAX_RES),
        ("dtype", c_int32),
    ]


def make_mrf_config(channels, resblock_kernel_sizes, resblock_dilation_sizes,
                    precision: str = "fp32") -> HfgMrfConfig:
    """One MRF's hyper-parameters (MRF.__init__, models/hifigan.py:96-114)."""
    n = min(len(resblock_kernel_sizes), len(resblock_dilation_sizes))  # zip semantics
    if n > HFG_MAX_RES:
        raise ValueError("too many resblocks for the ABI")
    c = HfgMrfConfig()
    c.channels = int(channels)
    c.n_res = n
    for j in range(n):
        dils = list(resblock_dilation_sizes[j])
        if len(dils) > HFG_MAX_DIL:
            raise ValueError("too many dilations in one ResBlock")
        c.res_kernels[j] = int(resblock_kernel_sizes[j])
        c.n_dil[j] = len(dils)
        for m, d in enumerate(dils):
            c.dil[j][m] = int(d)
    if precision not in DTYPES:
        raise ValueError(f"precision must be one of {sorted(DTYPES)}")
    c.dtype = DTYPES[precision]
    return c


def make_config(n_mels, upsample_rates, upsample_kernel_sizes, upsample_initial_channel,
                resblock_kernel_sizes, resblock_dilation_sizes, precision: str = "fp32") -> HfgConfig:
    if len(upsample_rates) != len(upsample_kernel_sizes):
        raise ValueError("upsample_rates and upsample_kernel_sizes differ in length")
    if len(resblock_kernel_sizes) != len(resblock_dilation_sizes):
        # the reference zips them (models/hifigan.py:106); keep its truncation semantics
        n = min(len(resblock_kernel_sizes), len(resblock_dilation_sizes))
        resblock_kernel_sizes = list(resblock_kernel_sizes)[:n]
        resblock_dilation_sizes = list(resblock_dilation_sizes)[:n]
    if len(upsample_rates) > HFG_MAX_STAGES or len(resblock_kernel_sizes) > HFG_MAX_RES:
        raise ValueError("configuration exceeds the ABI's stage / resblock limits")
    c = HfgConfig()
    c.n_mels = int(n_mels)
    c.n_up = len(upsample_rates)
    for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
        c.up_rates[i] = int(u)
        c.up_kernels[i] = int(k)
    c.c0 = int(upsample_initial_channel)
    c.n_res = len(resblock_kernel_sizes)
    for j, (k, dils) in enumerate(zip(resblock_kernel_sizes, resblock_dilation_sizes)):
        if len(dils) > HFG_MAX_DIL:
            raise ValueError("too many dilations in one ResBlock")
        c.res_kernels[j] = int(k)
        c.n_dil[j] = len(dils)
        for m, d in enumerate(dils):
            c.dil[j][m] = int(d)
    if precision not in DTYPES:
        raise ValueError(f"precision must be one of {sorted(DTYPES)}")
    c.dtype = DTYPES[precision]
    return c


class HfgMelConfig(ctypes.Structure):
    _fields_ = [("sample_rate", c_int32), ("n_fft", c_int32), ("hop_length", c_int32),
                ("win_length", c_int32), ("n_mels", c_int32), ("f_min", c_float),
                ("f_max", c_float), ("mel_scale", c_int32), ("norm", c_int32),
                ("log_eps", c_float), ("log_base", c_int32), ("log_base_value", c_float)]


_lib = None

# name -> (restype, argtypes); every symbol declared in include/hifigan_hip*.h
SIGNATURES = {
    "hfg_version": (c_char_p, []),
    "hfg_last_error": (c_char_p, []),
    "hfg_create": (c_int, [POINTER(HfgConfig), c_int, POINTER(c_void_p)]),
    "hfg_destroy": (None, [c_void_p]),
    "hfg_num_params": (c_int, [c_void_p]),
    "hfg_set_weight": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int, c_int]),
    "hfg_commit_weights": (c_int, [c_void_p]),
    "hfg_out_len": (c_int64, [c_void_p, c_int64]),
    "hfg_workspace_bytes": (c_size_t, [c_void_p, c_int64, c_int64]),
    "hfg_reserve": (c_int, [c_void_p, c_int64, c_int64]),
    "hfg_forward": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p]),
    "hfg_forward_ws": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64,
                               c_void_p, c_size_t, c_void_p]),
    "hfg_forward_ex": (c_int, [c_void_p, c_void_p, c_int64, c_int64, POINTER(HfgForwardOpts),
                               c_void_p, c_int64, c_void_p, c_size_t, c_void_p]),
    "hfg_set_profiling": (c_int, [c_void_p, c_int]),
    "hfg_set_streams": (c_int, [c_void_p, c_int]),
    "hfg_profile_reset": (c_int, [c_void_p]),
    "hfg_profile_summary": (c_int, [c_void_p, c_char_p, c_size_t]),
    "hfg_debug_packed_layer": (c_int, [c_void_p, c_char_p, POINTER(c_float), c_size_t,
                                       POINTER(c_int64)]),
    "hfg_debug_layer_exponent": (c_int, [c_void_p, c_char_p, POINTER(c_int)]),
    "hfg_debug_packed_resblock": (c_int, [c_void_p, c_int, c_int, POINTER(c_float), c_size_t,
                                          POINTER(c_int64)]),
    "hfg_mrf_create": (c_int, [POINTER(HfgMrfConfig), c_int, POINTER(c_void_p)]),
    "hfg_mrf_workspace_bytes": (c_size_t, [c_void_p, c_int64, c_int64]),
    "hfg_mrf_forward": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                c_size_t, c_void_p]),
    "hfg_resblock_forward": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_void_p,
                                     c_void_p, c_size_t, c_void_p]),
    "hfg_checksum32": (c_int, [POINTER(c_void_p), POINTER(c_int64), c_int, c_void_p, c_void_p]),
    "hfg_forward_taps": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int64,
                                 c_void_p, c_size_t, POINTER(c_void_p), c_int, c_void_p]),
    "hfg_probe_mfma_rate": (c_int, [c_int, c_int, c_int, POINTER(c_double), POINTER(c_double)]),
    "hfg_debug_schedule_set": (c_int, [c_char_p, c_int]),
    "hfg_debug_schedule_clear": (c_int, [c_char_p]),
    "hfg_debug_schedule_get": (c_int, [c_char_p, POINTER(c_int)]),
    "hfg_mel_last_error": (c_char_p, []),
    "hfg_mel_create": (c_int, [POINTER(HfgMelConfig), c_int, POINTER(c_void_p)]),
    "hfg_mel_destroy": (None, [c_void_p]),
    "hfg_mel_filterbank": (c_int, [POINTER(HfgMelConfig), POINTER(c_float)]),
    "hfg_mel_set_tables": (c_int, [c_void_p, POINTER(c_float), POINTER(c_float)]),
    "hfg_mel_frames": (c_int64, [c_void_p, c_int64]),
    "hfg_mel_workspace_bytes": (c_size_t, [c_void_p, c_int64, c_int64]),
    "hfg_mel_forward": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                c_size_t, c_void_p]),
    "hfg_resample_kernel": (c_int, [c_int32, c_int32, c_int32, c_float, POINTER(c_float),
                                    POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "hfg_resample_create": (c_int, [c_int32, c_int32, c_int32, c_float, c_int, POINTER(c_void_p)]),
    "hfg_resample_destroy": (None, [c_void_p]),
    "hfg_resample_out_len": (c_int64, [c_void_p, c_int64]),
    "hfg_resample_forward": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
}


def load_library(path: str = LIB_PATH):
    """Open libhifigan_hip.so (cached).  Raises HipExtensionMissing if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HipExtensionMissing(
            f"{path} is missing: the HIP extension must be built first "
            "(python tts-sambert_hifigan_amd/build.py). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    # a library missing an entry point is stale: refuse it, unless the caller
    # opts in for a same-box A/B against a previous commit's build (HFG_ALLOW_OLD_LIB=1)
    allow_old = os.environ.get("HFG_ALLOW_OLD_LIB") == "1"
    missing = []
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing and not allow_old:
        raise HipExtensionMissing(
            f"{path} lacks {', '.join(missing)}: it was built from an older tree; rebuild it "
            "(python tts-sambert_hifigan_amd/build.py) or set HFG_ALLOW_OLD_LIB=1 for an A/B")
    _lib = lib
    return lib


def library_source_hash(lib=None) -> str:
    """The source-tree hash compiled into the loaded library (hfg_version "src:...")."""
    v = (lib or load_library()).hfg_version().decode()
    return v.rsplit("src:", 1)[-1] if "src:" in v else ""


def check_provenance(lib=None) -> str:
    """Raise unless the loaded libhifigan_hip.so was built from THIS tree's csrc/ and
    include/ (the sha256 build.py computes over them == the one compiled into
    hfg_version).  Returns the hash.  Used by smoke() and the GPU test session."""
    from .build import source_hash
    want, got = source_hash(), library_source_hash(lib)
    if want != got:
        raise HipExtensionMissing(
            f"{LIB_PATH} was built from source tree {got or '?'}, this tree is {want}: "
            "rebuild it (python tts-sambert_hifigan_amd/build.py)")
    return got


def check(rc: int):
    if rc != 0:
        msg = load_library().hfg_last_error().decode(errors="replace")
        raise HfgError(rc, msg)
    return rc


def schedule_override(knob: str, value: int):
    """Force one schedule choice for every handle created afterwards in this process
    (hfg_debug_schedule_set, include/hifigan_hip_inspect.h): A/B runs and the parity suites'
    forced paths.  The library never reads its schedule from the environment."""
    check(load_library().hfg_debug_schedule_set(knob.encode(), int(value)))


def schedule_clear(knob: Optional[str] = None):
    """Drop one override (or all): later handles run the default schedule."""
    check(load_library().hfg_debug_schedule_clear(None if knob is None else knob.encode()))


def schedule_overrides() -> dict:
    """The overrides in force, {knob: value}."""
    lib = load_library()
    out = {}
    for k in ("FUSED_RB", "FUSE_POST", "RB_SPLIT", "SMALL_TILE", "RB_CONC", "UPS_FRAMES", "SPLIT",
              "RB_PERSIST", "DEBUG_FLAGS", "MEL_DFT", "AREG_TALL"):
        v = c_int(0)
        if lib.hfg_debug_schedule_get(k.encode(), ctypes.byref(v)) == 1:
            out[k] = v.value
    return out


def checksum32(tensors) -> "torch.Tensor":
    """Content hash per fp32 device tensor (hfg_checksum32) as an int64 CPU tensor.
    Synchronises with the current stream (the result is copied to the host)."""
    if not tensors:
        return torch.zeros(0, dtype=torch.int64)
    lib = load_library()
    dev = tensors[0].device
    n = len(tensors)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ptrs = (c_void_p * n)(*[t.data_ptr() for t in tensors])
    nbytes = (c_int64 * n)(*[t.numel() * t.element_size() for t in tensors])
    check(lib.hfg_checksum32(ptrs, nbytes, n, c_void_p(out.data_ptr()),
                             c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return out.cpu().to(torch.int64)


class Handle:
    """Owning wrapper of an ``hfg_handle*`` (one per device): a Generator handle
    (``hfg_create``) or, with ``mrf=True``, an MRF handle (``hfg_mrf_create``)."""

    def __init__(self, cfg, device: int, mrf: bool = False):
        self.lib = load_library()
        self.device = device
        self.mrf = mrf
        h = c_void_p()
        create = self.lib.hfg_mrf_create if mrf else self.lib.hfg_create
        check(create(ctypes.byref(cfg), int(device), ctypes.byref(h)))
        self.ptr = h

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.lib.hfg_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass

    def set_weight(self, name: str, t: "torch.Tensor"):
        """Copy one parameter in (hfg_set_weight).  A device tensor is first ordered
        after the producing work on torch's current stream (the library's D2H copy
        runs on the null stream)."""
        t = t.detach()
        is_dev = 1 if t.is_cuda else 0
        t = t.to(torch.float32).contiguous()
        if is_dev:
            torch.cuda.current_stream(t.device).synchronize()
        shape = (c_int64 * max(t.dim(), 1))(*t.shape)
        check(self.lib.hfg_set_weight(self.ptr, name.encode(), c_void_p(t.data_ptr()), shape,
                                      t.dim(), is_dev))

    def commit(self):
        check(self.lib.hfg_commit_weights(self.ptr))

    def out_len(self, T: int) -> int:
        return int(self.lib.hfg_out_len(self.ptr, int(T)))

    def workspace_bytes(self, B: int, T: int) -> int:
        return int(self.lib.hfg_workspace_bytes(self.ptr, int(B), int(T)))

    def forward_ws(self, mel_ptr: int, B: int, T: int, wav_ptr: int, out_len: int, ws_ptr: int,
                   ws_bytes: int, stream: int):
        check(self.lib.hfg_forward_ws(self.ptr, c_void_p(mel_ptr), int(B), int(T),
                                      c_void_p(wav_ptr), int(out_len), c_void_p(ws_ptr),
                                      int(ws_bytes), c_void_p(stream)))

    def forward_ex(self, mel_ptr: int, B: int, T: int, wav_ptr: int, out_len: int, ws_ptr: int,
                   ws_bytes: int, stream: int, mel_layout: str = "bct", lengths_ptr: int = 0):
        o = HfgForwardOpts(MEL_LAYOUTS[mel_layout], c_void_p(lengths_ptr) if lengths_ptr else None)
        check(self.lib.hfg_forward_ex(self.ptr, c_void_p(mel_ptr), int(B), int(T), ctypes.byref(o),
                                      c_void_p(wav_ptr), int(out_len), c_void_p(ws_ptr),
                                      int(ws_bytes), c_void_p(stream)))

    def forward_taps(self, mel_ptr: int, B: int, T: int, wav_ptr: int, out_len: int, ws_ptr: int,
                     ws_bytes: int, tap_ptrs, stream: int):
        n = len(tap_ptrs)
        arr = (c_void_p * n)(*[p if p else None for p in tap_ptrs])
        check(self.lib.hfg_forward_taps(self.ptr, c_void_p(mel_ptr), int(B), int(T),
                                        c_void_p(wav_ptr), int(out_len), c_void_p(ws_ptr),
                                        int(ws_bytes), arr, n, c_void_p(stream)))

    def mrf_workspace_bytes(self, B: int, L: int) -> int:
        return int(self.lib.hfg_mrf_workspace_bytes(self.ptr, int(B), int(L)))

    def mrf_forward(self, x_ptr: int, B: int, L: int, y_ptr: int, ws_ptr: int, ws_bytes: int,
                    stream: int, resblock: int = -1):
        if resblock < 0:
            check(self.lib.hfg_mrf_forward(self.ptr, c_void_p(x_ptr), int(B), int(L),
                                           c_void_p(y_ptr), c_void_p(ws_ptr), int(ws_bytes),
                                           c_void_p(stream)))
        else:
            check(self.lib.hfg_resblock_forward(self.ptr, int(resblock), c_void_p(x_ptr), int(B),
                                                int(L), c_void_p(y_ptr), c_void_p(ws_ptr),
                                                int(ws_bytes), c_void_p(stream)))

    def set_streams(self, n: int):
        """1: every launch on the caller's stream; 2: batch halves on two streams."""
        check(self.lib.hfg_set_streams(self.ptr, int(n)))

    def set_profiling(self, on: bool):
        check(self.lib.hfg_set_profiling(self.ptr, 1 if on else 0))

    def profile_reset(self):
        check(self.lib.hfg_profile_reset(self.ptr))

    def profile_summary(self) -> dict:
        import json
        buf = ctypes.create_string_buffer(1 << 16)
        check(self.lib.hfg_profile_summary(self.ptr, buf, len(buf)))
        return json.loads(buf.value.decode())

    def packed_layer(self, mod: str):
        """(info dict, packed weights np.ndarray, per-row bias np.ndarray) of one layer."""
        import numpy as np
        info = (c_int64 * 10)()
        check(self.lib.hfg_debug_packed_layer(self.ptr, mod.encode(), None, 0, info))
        w_len, b_len = int(info[6]), int(info[7])
        out = np.zeros(w_len + b_len, dtype=np.float32)
        check(self.lib.hfg_debug_packed_layer(
            self.ptr, mod.encode(), out.ctypes.data_as(POINTER(c_float)), out.size, info))
        ew = c_int(0)
        check(self.lib.hfg_debug_layer_exponent(self.ptr, mod.encode(), ctypes.byref(ew)))
        keys = ["kind", "M", "KT", "tile", "m_tiles", "n_chunks", "w_len", "b_len", "CK", "MT"]
        d = dict(zip(keys, [int(v) for v in info]))
        d["ew"] = int(ew.value)
        return d, out[:w_len], out[w_len:]

    def packed_resblock(self, stage: int, j: int):
        """(info dict, packed A stream, biases) of a whole-ResBlock launch, or
        (info with fused=0, None, None) when the stage runs layer by layer."""
        import numpy as np
        info = (c_int64 * 8)()
        check(self.lib.hfg_debug_packed_resblock(self.ptr, stage, j, None, 0, info))
        keys = ["fused", "C", "KT", "n_conv", "halo", "W", "w_len", "b_len"]
        d = dict(zip(keys, [int(v) for v in info]))
        if not d["fused"]:
            return d, None, None
        out = np.zeros(d["w_len"] + d["b_len"], dtype=np.float32)
        check(self.lib.hfg_debug_packed_resblock(
            self.ptr, stage, j, out.ctypes.data_as(POINTER(c_float)), out.size, info))
        return d, out[:d["w_len"]], out[d["w_len"]:]

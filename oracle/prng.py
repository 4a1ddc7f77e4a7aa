"""Portable counter-based PRNG for reproducible Generator weights and mel inputs.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Element ``i`` of the stream keyed by ``(seed, name)`` is
``splitmix64_mix(key + (i + 1) * GOLDEN)`` with ``key = fnv1a64(name) ^ mix(seed)``.
Everything is exact integer / IEEE arithmetic, so numpy, C and any other
language produce bit-identical streams.

Weight bounds restate PyTorch's default init for the modules the reference
builds (``models/hifigan.py:177-222`` → ``nn.Conv1d`` / ``nn.ConvTranspose1d``
``reset_parameters``: kaiming_uniform(a=sqrt(5)) ⇒ U(±1/sqrt(fan_in)) for the
weight and the bias, fan_in = ``weight.size(1) * k``).
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def stream_key(seed: int, name: str) -> np.uint64:
    s = _mix(np.array([seed & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))[0]
    return np.uint64(fnv1a64(name)) ^ s


def uniform01(seed: int, name: str, n: int) -> np.ndarray:
    """n float64 values in [0, 1) with 53-bit resolution."""
    key = stream_key(seed, name)
    idx = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _mix(key + idx * GOLDEN)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def uniform_sym(seed: int, name: str, shape, bound: float) -> np.ndarray:
    """float32 U(-bound, bound) of the given shape."""
    n = int(np.prod(shape))
    u = uniform01(seed, name, n)
    return ((2.0 * u - 1.0) * bound).astype(np.float32).reshape(shape)


def normal(seed: int, name: str, shape, std: float = 1.0) -> np.ndarray:
    """float32 N(0, std^2) by Box-Muller on two keyed uniform streams."""
    n = int(np.prod(shape))
    u1 = uniform01(seed, name + "#bm1", n)
    u2 = uniform01(seed, name + "#bm2", n)
    r = np.sqrt(-2.0 * np.log1p(-u1))  # 1-u1 in (0, 1]
    return (r * np.cos(2.0 * np.pi * u2) * std).astype(np.float32).reshape(shape)


def mel_input(seed: int, shape) -> np.ndarray:
    """Synthetic log-mel input [B, n_mels, T] ~ N(0, 1) (values do not affect speed)."""
    return normal(seed, "mel", shape)

"""Deterministic synthetic audio (SURVEY.md §8d "Synthetic inputs").

No datasets are reachable offline, so every benchmark / parity input is generated here from a seed:
f32 mono 16 kHz, peak-normalised to 0.5, a "speech-like" signal (3 harmonics, f0 wandering
100-250 Hz, 4 Hz syllable AM, 300 ms silences every ~3 s) plus N(0, 0.01^2) noise.
"""
from __future__ import annotations

import hashlib

import numpy as np

SAMPLE_RATE = 16000


def speech_like(seed: int, n_samples: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples, dtype=np.float64) / SAMPLE_RATE
    phi = rng.uniform(0, 2 * np.pi, size=3)
    f0 = 175.0 + 75.0 * np.sin(2 * np.pi * 0.3 * t + phi[0])
    phase = 2 * np.pi * np.cumsum(f0) / SAMPLE_RATE
    amps = rng.uniform(0.3, 1.0, size=3)
    x = sum(a * np.sin((h + 1) * phase + phi[h]) for h, a in enumerate(amps))
    am = 0.55 + 0.45 * np.sin(2 * np.pi * 4.0 * t + phi[1])
    gate = np.ones(n_samples)
    period = int(3.0 * SAMPLE_RATE)
    gap = int(0.3 * SAMPLE_RATE)
    start = int(rng.integers(0, period))
    for s in range(start, n_samples, period):
        gate[s: s + gap] = 0.0
    x = x * am * gate + rng.normal(0.0, 0.01, size=n_samples)
    peak = np.max(np.abs(x)) if n_samples else 0.0
    if peak > 0:
        x = x * (0.5 / peak)
    return x.astype(np.float32)


def white_noise(seed: int, n_samples: int, sigma: float = 0.1) -> np.ndarray:
    return np.random.default_rng(seed).normal(0.0, sigma, size=n_samples).astype(np.float32)


def digest(x: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(x, dtype=np.float32).tobytes()).hexdigest()

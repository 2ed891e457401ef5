"""Portable, counter-based synthetic data for the adaptive-attention decode path.

The reference initialises its weights with torch's CPU RNG, LAPACK QR (``orthogonal_``) and a
construction order that includes a throw-away baseline ``AdaptiveBlock``
(``code_src/models/baseline_attention.py:143``, ``code_src/models/adaptive_attention.py:155``),
so "the same random-init weights" cannot be reproduced on another host from a seed.  This module
replaces the RNG with splitmix64 over a (key, element index) counter: every value is a pure
function of integers, computed with IEEE-exact float64 arithmetic and one round-to-nearest cast to
fp32.  The same formulas run on the GPU (``aa_synth_fill`` in ``csrc/aa_synth.hip``) and give the
same bits, so a GPU box regenerates identical weights and features without the reference.

Distributions follow ``code_src/models/model_utils.py:4-74`` (bounds/std from the init gains):

* ``xavier_uniform(gain)``      : U(-b, b), b = gain * sqrt(6 / (fan_in + fan_out))    (:4-16)
* ``kaiming_uniform('relu')``   : U(-b, b), b = sqrt(6 / fan_in)                        (:34-45)
* ``kaiming_normal('relu')``    : N(0, 2 / fan_in)                                      (:48-59)
* ``orthogonal_`` (LSTM)        : replaced by U with the variance of an orthonormal-column
                                  matrix, 1 / max(rows, cols)                            (:62-74)
* ``nn.Embedding`` default      : N(0, 1) (the reference never re-initialises ``embed``)
* biases                        : 0, LSTM forget slice [H:2H] = 0.5 in both bias vectors (:69-71)

Normals are Irwin-Hall(4) sums of 24-bit uniforms (variance-matched, no transcendental, so no
libm or SIMD-dispatch dependence).
"""
from __future__ import annotations

import hashlib
import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

MASK64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
MIX1 = 0xBF58476D1CE4E5B9
MIX2 = 0x94D049BB133111EB
INV24 = 1.0 / (1 << 24)

FEAT_SEED_DEFAULT = 0
WEIGHT_SEED_DEFAULT = 123


def _mix_int(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * MIX1) & MASK64
    z = ((z ^ (z >> 27)) * MIX2) & MASK64
    return z ^ (z >> 31)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h = ((h ^ b) * 0x100000001B3) & MASK64
    return h


def stream_key(seed: int, name: str) -> int:
    """64-bit key of one named stream (a weight tensor or the feature map)."""
    return _mix_int((seed * GOLDEN + fnv1a64(name)) & MASK64)


def uniform24(key: int, start: int, n: int) -> np.ndarray:
    """u[i] = (splitmix64(key + (start+i+1)*GOLDEN) >> 40) / 2^24 as float64 (exact), i < n."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(key) + i * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(MIX1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(MIX2)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) * INV24


def uniform_f32(key: int, start: int, n: int, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """fp32(lo + (hi - lo) * u): for lo=0, hi=1 the value is u itself, exactly."""
    u = uniform24(key, start, n)
    if lo == 0.0 and hi == 1.0:
        return u.astype(np.float32)
    return (lo + (hi - lo) * u).astype(np.float32)


def symmetric_f32(key: int, n: int, bound: float) -> np.ndarray:
    """U(-bound, bound): fp32((2u - 1) * bound)."""
    return ((2.0 * uniform24(key, 0, n) - 1.0) * float(bound)).astype(np.float32)


def normal_f32(key: int, n: int, std: float) -> np.ndarray:
    """Irwin-Hall(4) normal: fp32((u0+u1+u2+u3 - 2) * sqrt(3) * std); counters 4i..4i+3."""
    u = uniform24(key, 0, 4 * n).reshape(n, 4)
    s = ((u[:, 0] + u[:, 1]) + u[:, 2]) + u[:, 3]
    return ((s - 2.0) * (math.sqrt(3.0) * float(std))).astype(np.float32)


@dataclass(frozen=True)
class Dims:
    """Model dimensions (``code_src/config/cfg_wzn.py:115-116``, vocab.pkl length 10123)."""

    embed: int = 256      # cf.adaptive_word_embed_size
    hidden: int = 512     # cf.adaptive_lstm_hidden_size
    vocab: int = 10123    # cf.vocab_length = len(vocab.pkl)
    channels: int = 2048  # ResNet-152 last conv channels (baseline_attention.py:22-23)
    spatial: int = 49     # 7x7 locations == attention width (adaptive_attention.py:16-19)


def weight_specs(d: Dims) -> List[Tuple[str, Tuple[int, ...], str, float]]:
    """(state-dict key, shape, kind, scale) for every parameter of the adaptive Encoder2Decoder.

    Keys and shapes mirror the reference module tree: ``AttentiveCNN`` (baseline_attention.py:11-34),
    ``Decoder`` (baseline_attention.py:132-146 + adaptive_attention.py:151-155),
    ``AdaptiveBlock`` (adaptive_attention.py:89-108), ``Sentinel`` (:62-73), ``Atten`` (:12-24).
    """
    H, E, V, C, P = d.hidden, d.embed, d.vocab, d.channels, d.spatial
    g_tanh = 5.0 / 3.0
    kai_u = lambda fan_in: math.sqrt(6.0 / fan_in)
    xav_u = lambda gain, fi, fo: gain * math.sqrt(6.0 / (fi + fo))
    ortho = lambda r, c: math.sqrt(3.0 / max(r, c))
    return [
        ("encoder.affine_a.weight", (H, C), "uniform", kai_u(C)),
        ("encoder.affine_a.bias", (H,), "zero", 0.0),
        ("encoder.affine_b.weight", (E, C), "uniform", kai_u(C)),
        ("encoder.affine_b.bias", (E,), "zero", 0.0),
        ("encoder.affine_h0.weight", (H, C), "uniform", xav_u(g_tanh, C, H)),
        ("encoder.affine_h0.bias", (H,), "zero", 0.0),
        ("encoder.affine_c0.weight", (H, C), "uniform", xav_u(g_tanh, C, H)),
        ("encoder.affine_c0.bias", (H,), "zero", 0.0),
        ("decoder.embed.weight", (V, E), "normal", 1.0),
        ("decoder.LSTM.weight_ih_l0", (4 * H, 2 * E), "uniform", ortho(4 * H, 2 * E)),
        ("decoder.LSTM.weight_hh_l0", (4 * H, H), "uniform", ortho(4 * H, H)),
        ("decoder.LSTM.bias_ih_l0", (4 * H,), "lstm_bias", 0.0),
        ("decoder.LSTM.bias_hh_l0", (4 * H,), "lstm_bias", 0.0),
        ("decoder.adaptive.sentinel.affine_x.weight", (H, 2 * E), "uniform", xav_u(1.0, 2 * E, H)),
        ("decoder.adaptive.sentinel.affine_h.weight", (H, H), "uniform", xav_u(1.0, H, H)),
        ("decoder.adaptive.atten.affine_v.weight", (P, H), "uniform", xav_u(g_tanh, H, P)),
        ("decoder.adaptive.atten.affine_g.weight", (P, H), "uniform", xav_u(g_tanh, H, P)),
        ("decoder.adaptive.atten.affine_s.weight", (P, H), "uniform", xav_u(g_tanh, H, P)),
        ("decoder.adaptive.atten.affine_h.weight", (1, P), "normal", math.sqrt(2.0 / P)),
        ("decoder.adaptive.mlp.weight", (V, H), "normal", math.sqrt(2.0 / H)),
        ("decoder.adaptive.mlp.bias", (V,), "zero", 0.0),
    ]


def make_weights(seed: int = WEIGHT_SEED_DEFAULT, d: Dims = Dims(), bias_noise: float = 0.0) -> Dict[str, np.ndarray]:
    """Deterministic state dict (fp32 numpy).  ``bias_noise > 0`` adds U(-n, n) to every bias so
    parity tests also exercise the bias paths (the reference init zeroes them)."""
    out: Dict[str, np.ndarray] = {}
    H = d.hidden
    for name, shape, kind, scale in weight_specs(d):
        n = int(np.prod(shape))
        key = stream_key(seed, name)
        if kind == "uniform":
            w = symmetric_f32(key, n, scale)
        elif kind == "normal":
            w = normal_f32(key, n, scale)
        elif kind == "zero":
            w = np.zeros(n, np.float32)
        elif kind == "lstm_bias":
            w = np.zeros(n, np.float32)
            w[H:2 * H] = 0.5
        else:  # pragma: no cover
            raise ValueError(kind)
        if bias_noise and name.rsplit(".", 1)[-1].startswith("bias"):
            w = (w.astype(np.float64) + (2.0 * uniform24(stream_key(seed, name + "#noise"), 0, n) - 1.0) * bias_noise).astype(np.float32)
        out[name] = w.reshape(shape)
    return out


def make_features(B: int, seed: int = FEAT_SEED_DEFAULT, row0: int = 0, d: Dims = Dims()) -> np.ndarray:
    """Post-trunk ResNet features [B, C, 7, 7] (NCHW, what ``AttentiveCNN.forward`` sees after
    ``resnet_conv``, baseline_attention.py:43), U[0,1) fp32.  Element (b, c, p) of global row
    ``row0 + b`` is counter ``((row0+b) * C + c) * 49 + p``, so a rank-sharded batch reproduces
    the rows of the full batch exactly."""
    C, P = d.channels, d.spatial
    per_row = C * P
    key = stream_key(seed, "features")
    x = uniform_f32(key, row0 * per_row, B * per_row)
    return x.reshape(B, C, 7, 7)


def digest(arrays: Dict[str, np.ndarray]) -> Dict[str, str]:
    return {k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() for k, v in arrays.items()}

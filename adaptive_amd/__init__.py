"""adaptive_amd — MI355X-native greedy decode of the adaptive-attention captioner.

The hot path of wzn0828/Adaptive (``Encoder2Decoder.sampler``, code_src/models/adaptive_attention.py)
rebuilt as hand-written gfx950 HIP kernels behind a C-ABI (include/adaptive_amd.h), bound here with
ctypes and wrapped in a drop-in ``Encoder2Decoder`` module.
"""
from .synth import Dims, make_features, make_weights  # noqa: F401

__all__ = ["Dims", "make_features", "make_weights", "Encoder2Decoder", "Config", "DecodePlan"]


def __getattr__(name):  # lazy: importing the package must not require torch/HIP
    if name in ("Encoder2Decoder", "Config", "synthetic_features", "DecodePlan"):
        from . import adaptive_attention
        return getattr(adaptive_attention, name)
    raise AttributeError(name)

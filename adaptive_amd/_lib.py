"""ctypes binding of the C-ABI in ``include/adaptive_amd.h`` (``libadaptive_amd.so``).

``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and the kernel
library must bind to that same HIP runtime (one runtime per process).  There
is no CPU fallback: a missing or unloadable library raises ``RuntimeError`` with the build
command.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from ctypes import POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_uint64, c_void_p

import torch  # noqa: F401  (must precede the CDLL: shares torch's HIP runtime)

# AA_LIB_PATH: load another build of the same library (A/B timing of two builds in one GPU session)
LIB_PATH = os.environ.get("AA_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                         "libadaptive_amd.so")
ABI_VERSION = 16
DECODE_EXACT_VOCAB = 1
DECODE_FP32_ENCODER = 2
DECODE_ONE_STREAM = 512
DECODE_SPLIT_RESCORE = 1024  # rescoring in its own launch per step (cross-check of the fused default)
DECODE_RS_SELF = 2048  # test hook: fused launch's LSTM workgroups rescore unpublished rows themselves
DECODE_SCREEN4 = 4096  # vocab screen on k_vscreen2 (4 waves) instead of k_vscreen8: the same summaries
BEAM_FAST = 256
TRAIN_BF16 = 128
MAX_BEAM = 8


class Dims(Structure):
    _fields_ = [("embed", c_int32), ("hidden", c_int32), ("vocab", c_int32), ("channels", c_int32), ("spatial", c_int32)]


# aa_ref_weights field  <->  reference state-dict key
WEIGHT_FIELDS = [
    ("enc_affine_a_w", "encoder.affine_a.weight"),
    ("enc_affine_a_b", "encoder.affine_a.bias"),
    ("enc_affine_b_w", "encoder.affine_b.weight"),
    ("enc_affine_b_b", "encoder.affine_b.bias"),
    ("enc_affine_h0_w", "encoder.affine_h0.weight"),
    ("enc_affine_h0_b", "encoder.affine_h0.bias"),
    ("enc_affine_c0_w", "encoder.affine_c0.weight"),
    ("enc_affine_c0_b", "encoder.affine_c0.bias"),
    ("embed_w", "decoder.embed.weight"),
    ("lstm_w_ih", "decoder.LSTM.weight_ih_l0"),
    ("lstm_w_hh", "decoder.LSTM.weight_hh_l0"),
    ("lstm_b_ih", "decoder.LSTM.bias_ih_l0"),
    ("lstm_b_hh", "decoder.LSTM.bias_hh_l0"),
    ("sent_affine_x_w", "decoder.adaptive.sentinel.affine_x.weight"),
    ("sent_affine_h_w", "decoder.adaptive.sentinel.affine_h.weight"),
    ("att_affine_v_w", "decoder.adaptive.atten.affine_v.weight"),
    ("att_affine_g_w", "decoder.adaptive.atten.affine_g.weight"),
    ("att_affine_s_w", "decoder.adaptive.atten.affine_s.weight"),
    ("att_affine_h_w", "decoder.adaptive.atten.affine_h.weight"),
    ("mlp_w", "decoder.adaptive.mlp.weight"),
    ("mlp_b", "decoder.adaptive.mlp.bias"),
]


class RefWeights(Structure):
    _fields_ = [(f, c_void_p) for f, _ in WEIGHT_FIELDS]


class Model(Structure):
    _fields_ = [("dims", Dims), ("packed", c_void_p), ("packed_bytes", c_size_t)]


TRACE_ENCODER_KERNELS = 5  # k_avgpool, k_enc_v, k_enc_heads, VWv GEMM, x_g GEMM


class AdamTensor(Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("numel", c_int64)]


ADAM_MAX_TENSORS = 24


class GradTensor(Structure):
    _fields_ = [("grad", c_void_p), ("numel", c_int64)]


CLIP_MAX_TENSORS = 24


class Trace(Structure):
    _fields_ = [("encoder_events", c_void_p), ("lstm_events", c_void_p), ("atten_events", c_void_p),
                ("screen_events", c_void_p), ("rescore_events", c_void_p), ("gemm_events", c_void_p)]


# name -> (restype, argtypes); mirrors include/adaptive_amd.h one to one
SIGNATURES = {
    "aa_abi_version": (c_int, []),
    "aa_error_string": (c_char_p, [c_int]),
    "aa_check_dims": (c_int, [POINTER(Dims)]),
    "aa_packed_bytes": (c_size_t, [POINTER(Dims)]),
    "aa_pack_weights": (c_int, [POINTER(Model), POINTER(RefWeights), c_void_p]),
    "aa_encoder_tail": (c_int, [POINTER(Model), c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_int32, c_void_p]),
    "aa_step_workspace_bytes": (c_size_t, [POINTER(Dims), c_int32]),
    "aa_decode_step": (c_int, [POINTER(Model), c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                               c_void_p]),
    "aa_decode_workspace_bytes": (c_size_t, [POINTER(Dims), c_int32, c_int32]),
    "aa_greedy_decode": (c_int, [POINTER(Model), c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_size_t, POINTER(Trace), c_int32, c_void_p]),
    "aa_greedy_decode_aux": (c_int, [POINTER(Model), c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size_t, POINTER(Trace), c_int32, c_void_p, c_void_p]),
    "aa_decode_plan_create": (c_int, [POINTER(Model), c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_size_t, c_int32, POINTER(c_void_p)]),
    "aa_decode_plan_launch": (c_int, [c_void_p, c_void_p]),
    "aa_decode_plan_destroy": (c_int, [c_void_p]),
    "aa_train_workspace_bytes": (c_size_t, [POINTER(Dims), c_int32, c_int32]),
    "aa_train_forward": (c_int, [POINTER(RefWeights), POINTER(Dims), c_void_p, c_int32, c_int32, c_void_p, c_int32,
                                 c_void_p, c_void_p, c_int32, c_void_p, c_size_t, c_int32, c_void_p]),
    "aa_train_backward": (c_int, [POINTER(RefWeights), POINTER(Dims), c_void_p, c_int32, c_int32, c_void_p, c_int32,
                                  c_void_p, c_void_p, c_int32, POINTER(RefWeights), c_void_p, c_void_p, c_size_t,
                                  c_int32, c_void_p]),
    "aa_train_forward_aux": (c_int, [POINTER(RefWeights), POINTER(Dims), c_void_p, c_int32, c_int32, c_void_p,
                                     c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_size_t, c_int32, c_void_p,
                                     c_void_p]),
    "aa_train_backward_aux": (c_int, [POINTER(RefWeights), POINTER(Dims), c_void_p, c_int32, c_int32, c_void_p,
                                      c_int32, c_void_p, c_void_p, c_int32, POINTER(RefWeights), c_void_p, c_void_p,
                                      c_size_t, c_int32, c_void_p, c_void_p]),
    "aa_decoder_workspace_bytes": (c_size_t, [POINTER(Dims), c_int32, c_int32]),
    "aa_decoder_forward": (c_int, [POINTER(RefWeights), POINTER(Dims), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                   c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_int32, c_void_p]),
    "aa_beam_workspace_bytes": (c_size_t, [POINTER(Dims), c_int32, c_int32, c_int32]),
    "aa_beam_decode": (c_int, [POINTER(Model), c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int32, c_void_p, c_void_p]),
    "aa_vocab_logits": (c_int, [POINTER(Model), c_int32, c_void_p, c_void_p, c_void_p]),
    "aa_vocab_logits_at": (c_int, [POINTER(Model), c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "aa_cross_entropy_workspace_bytes": (c_size_t, [c_int32]),
    "aa_cross_entropy_forward": (c_int, [c_void_p, c_int32, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                         c_void_p, c_size_t, c_void_p]),
    "aa_cross_entropy_backward": (c_int, [c_void_p, c_int32, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                          c_void_p, c_size_t, c_void_p, c_int64, c_void_p]),
    "aa_adam_step": (c_int, [POINTER(AdamTensor), c_int32, c_double, c_double, c_double, c_double, c_double,
                             c_double, c_void_p]),
    "aa_clip_grad_norm_workspace_bytes": (c_size_t, [POINTER(GradTensor), c_int32]),
    "aa_clip_grad_norm": (c_int, [POINTER(GradTensor), c_int32, c_float, c_void_p, c_void_p, c_size_t, c_void_p]),
    "aa_synth_uniform": (c_int, [c_void_p, c_int64, c_uint64, c_int64, c_double, c_double, c_void_p]),
    "aa_read_probe": (c_int, [c_void_p, c_size_t, c_void_p, c_int32, c_void_p]),
}

_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Load (once) and type the library.  Raises RuntimeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"adaptive_amd: HIP library not built ({LIB_PATH} missing). Build it with "
                "`make -C adaptive_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`. "
                "There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        partial = bool(os.environ.get("AA_LIB_PATH"))  # A/B builds may be greedy-only (AA_DECODE_ONLY)
        for name, (res, args) in SIGNATURES.items():
            if partial and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.aa_abi_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"adaptive_amd: ABI version {v} != expected {ABI_VERSION}; rebuild the library")
        _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().aa_error_string(rc).decode()
        raise RuntimeError(f"adaptive_amd{(' ' + what) if what else ''}: {msg} (code {rc})")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


_NO_SWITCH = contextlib.nullcontext()


def on_device(dev):
    """torch.cuda.device(dev), or a no-op context when `dev` is already the current device (the
    training step's calls make several per step; constructing the switch costs ≈ 6 us each)."""
    idx = dev.index if isinstance(dev, torch.device) else dev
    if idx is None or (_cur_device is not None and idx == _cur_device()):
        return _NO_SWITCH
    return torch.cuda.device(dev)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def stream_handle(stream=None) -> int:
    """The hipStream_t of `stream`, or of the current device's current stream -- read directly
    (torch.cuda.current_stream() builds a Stream object per call: ≈ 12 us, several times per training
    step)."""
    if stream is not None:
        return stream.cuda_stream
    if _raw_stream is not None and _cur_device is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream

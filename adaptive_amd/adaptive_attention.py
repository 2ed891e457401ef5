"""Drop-in ``Encoder2Decoder`` for the adaptive-attention model, executed by MI355X HIP kernels.

Mirrors the reference module tree and public surface so callers (``code_src/tools/utils.py:171``
``model.sampler(images)``, ``code_src/models/model_factory.py:10`` construction,
``code_src/train.py:177`` state-dict save) work unchanged:

* ``Encoder2Decoder(cf)``             — adaptive_attention.py:159-165
* ``.sampler(images, max_len=30)``   — adaptive_attention.py:168-216  -> (ids, alpha, beta)
* ``.encoder(images)``                — AttentiveCNN.forward, baseline_attention.py:36-62
* ``.decoder(V, v_g, captions, states)`` — Decoder.forward, baseline_attention.py:148-194
  (-> scores, alpha, beta, states): one-token captions run the sampling step, whole captions [B,T]
  the teacher-forced recurrence
* state-dict keys identical to the reference (``encoder.affine_a.weight``, ``decoder.LSTM.*``,
  ``decoder.adaptive.{sentinel,atten,mlp}.*``).

``images`` are the post-trunk ResNet-152 features [B, 2048, 7, 7] (the trunk,
baseline_attention.py:16-18, is out of scope: ``resnet_conv`` is an empty ``nn.Sequential``).
Parameters live in ordinary ``nn.Parameter``s; on first use after any change they are packed into
the kernel layout by ``aa_pack_weights``.  All compute goes through ``libadaptive_amd.so``; there
is no eager/CPU fallback — a CPU tensor or a missing library raises.

Reference defect D1 (``adaptive_attention.py:183,198`` passes [B,1,H] states to ``nn.LSTM`` and
raises for B > 1) is not reproduced: the sampler uses the baseline's transpose semantics
(``baseline_attention.py:251-252``).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.nn import init

from . import _lib
from .synth import Dims

ATT = 49


class Config:
    """The three ``cf`` attributes the path reads (cfg_wzn.py:115-116, train.py:40)."""

    def __init__(self, adaptive_word_embed_size: int = 256, adaptive_lstm_hidden_size: int = 512,
                 vocab_length: int = 10123):
        self.adaptive_word_embed_size = adaptive_word_embed_size
        self.adaptive_lstm_hidden_size = adaptive_lstm_hidden_size
        self.vocab_length = vocab_length


# ---- reference-style initialisers (model_utils.py:4-74) ------------------------------------------
def _xavier_uniform(nonlinearity, *mods):
    gain = init.calculate_gain(nonlinearity)
    for m in mods:
        init.xavier_uniform_(m.weight, gain)
        if m.bias is not None:
            m.bias.data.fill_(0)


def _kaiming(fn, nonlinearity, a, *mods):
    for m in mods:
        fn(m.weight, a=a, mode="fan_in", nonlinearity=nonlinearity)
        if m.bias is not None:
            m.bias.data.fill_(0)


def _lstm_init(lstm: nn.LSTM):
    H = lstm.hidden_size
    for name, p in lstm.named_parameters():
        if "bias" in name:
            init.constant_(p, 0.0)
            p.data[H:2 * H] = 0.5
        elif "weight" in name:
            init.orthogonal_(p)


class AttentiveCNN(nn.Module):
    """Encoder tail (baseline_attention.py:11-62) over post-trunk features."""

    def __init__(self, embed_size: int, hidden_size: int, cf=None, channels: int = 2048, trunk: bool = False):
        super().__init__()
        # ResNet-152 trunk (adaptive_amd/trunk.py) or, by default, identity over post-trunk features
        if trunk:
            from .trunk import resnet_conv
            self.resnet_conv = resnet_conv()
        else:
            self.resnet_conv = nn.Sequential()
        self.avgpool = nn.AvgPool2d(7)
        self.affine_a = nn.Linear(channels, hidden_size)
        self.affine_b = nn.Linear(channels, embed_size)
        self.dropout = nn.Dropout(0)
        _kaiming(init.kaiming_uniform_, "relu", 0, self.affine_a, self.affine_b)
        self.affine_h0 = nn.Linear(channels, hidden_size)
        self.affine_c0 = nn.Linear(channels, hidden_size)
        _xavier_uniform("tanh", self.affine_h0, self.affine_c0)
        self._owner = None  # set by Encoder2Decoder (weak back-reference for packing)

    def forward(self, images: torch.Tensor):
        """-> V [B,49,H], v_g [B,E], (h0, c0) each [B,1,H] (baseline_attention.py:43-62)."""
        owner = self._owner
        if owner is None:
            raise RuntimeError("AttentiveCNN must be used through Encoder2Decoder (it owns the packed weights)")
        return owner._encode(images)[:3]


class Atten(nn.Module):
    """Parameter holder of adaptive_attention.py:12-24."""

    def __init__(self, hidden_size: int, cf=None):
        super().__init__()
        self.affine_v = nn.Linear(hidden_size, ATT, bias=False)
        self.affine_g = nn.Linear(hidden_size, ATT, bias=False)
        self.affine_s = nn.Linear(hidden_size, ATT, bias=False)
        self.affine_h = nn.Linear(ATT, 1, bias=False)
        self.dropout = nn.Dropout(0)
        _xavier_uniform("tanh", self.affine_v, self.affine_g, self.affine_s)
        _kaiming(init.kaiming_normal_, "relu", 0, self.affine_h)


class Sentinel(nn.Module):
    """Parameter holder of adaptive_attention.py:62-73."""

    def __init__(self, input_size: int, hidden_size: int):
        super().__init__()
        self.affine_x = nn.Linear(input_size, hidden_size, bias=False)
        self.affine_h = nn.Linear(hidden_size, hidden_size, bias=False)
        self.dropout = nn.Dropout(0)
        _xavier_uniform("sigmoid", self.affine_x, self.affine_h)


class AdaptiveBlock(nn.Module):
    """Parameter holder of adaptive_attention.py:89-108."""

    def __init__(self, embed_size: int, hidden_size: int, vocab_size: int, cf=None):
        super().__init__()
        self.sentinel = Sentinel(embed_size * 2, hidden_size)
        self.atten = Atten(hidden_size, cf)
        self.mlp = nn.Linear(hidden_size, vocab_size)
        self.dropout = nn.Dropout(0)
        self.hidden_size = hidden_size
        _kaiming(init.kaiming_normal_, "relu", 0, self.mlp)


class Decoder(nn.Module):
    """Decoder (baseline_attention.py:132-194 + adaptive_attention.py:151-155)."""

    def __init__(self, embed_size: int, vocab_size: int, hidden_size: int, cf=None):
        super().__init__()
        self.embed = nn.Embedding(vocab_size, embed_size)
        self.LSTM = nn.LSTM(embed_size * 2, hidden_size, 1, batch_first=True)
        self.adaptive = AdaptiveBlock(embed_size, hidden_size, vocab_size, cf)
        _lstm_init(self.LSTM)
        self._owner = None

    def forward(self, V, v_g, captions, states=None):
        owner = self._owner
        if owner is None:
            raise RuntimeError("Decoder must be used through Encoder2Decoder (it owns the packed weights)")
        return owner._decode_step(V, v_g, captions, states)


class DecodePlan:
    """A greedy decode of fixed (B, max_len) captured once into a hipGraph (C-ABI
    ``aa_decode_plan_*``) over buffers the plan OWNS: its input ``images`` [B, C, 7, 7], its outputs
    ``ids`` / ``alpha`` / ``beta`` and its workspace.  ``plan(x)`` copies ``x`` into the plan's own
    input buffer (a device copy queued before the replay) and replays the graph; nothing of the
    caller's is retained, so freshly allocated batches (the reference's eval loop,
    code_src/tools/utils.py:167-171) never re-capture.  The outputs are the plan's buffers,
    overwritten by the next replay (``clone()`` them to keep them).  Replays are bit-identical to
    ``sampler``.  The plan binds the model's packed weights as they were when it was made; make a new
    plan after the weights change (``plan.valid_for(model)``)."""

    def __init__(self, model: "Encoder2Decoder", B: int, max_len: int = 30, exact_vocab: bool = False,
                 stream: Optional[torch.cuda.Stream] = None):
        B, T = int(B), int(max_len)
        if B <= 0 or T <= 0:
            raise ValueError(f"DecodePlan needs B > 0 and max_len > 0, got B={B}, max_len={T}")
        mstruct = model._model_struct()
        lib = self.lib = _lib.load()
        dev = self.device = model._packed.device
        d = model.dims
        self.B, self.T = B, T
        self.flags = (_lib.DECODE_EXACT_VOCAB if exact_vocab else 0) | model._decode_flags()
        if not getattr(model, "decode_aux_stream", False):  # one stream, as sampler (see _decode_into)
            self.flags |= _lib.DECODE_ONE_STREAM
        self._pack_ref = (model._packed.data_ptr(), model._pack_key)
        self._packed = model._packed  # the graph reads the packed weights: keep them alive
        self.stream = stream
        with torch.cuda.device(dev), torch.cuda.stream(stream or torch.cuda.current_stream(dev)):
            self.images = torch.empty(B, d.channels, 7, 7, dtype=torch.float32, device=dev)
            self.ids = torch.empty(B, T, dtype=torch.int64, device=dev)
            self.alpha = torch.empty(B, T, ATT, dtype=torch.float32, device=dev)
            self.beta = torch.empty(B, T, 1, dtype=torch.float32, device=dev)
            nbytes = lib.aa_decode_workspace_bytes(model._c_dims(), B, T)
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            h = ctypes.c_void_p()
            _lib.check(lib.aa_decode_plan_create(mstruct, self.images.data_ptr(), B, T, self.ids.data_ptr(),
                                                 self.alpha.data_ptr(), self.beta.data_ptr(), self.ws.data_ptr(),
                                                 nbytes, self.flags, ctypes.byref(h)), "decode_plan_create")
        self.handle = h
        self._done = None  # completion event of the last replay
        Encoder2Decoder._captures += 1

    def valid_for(self, model: "Encoder2Decoder") -> bool:
        return model._packed is not None and (model._packed.data_ptr(), model._pack_key) == self._pack_ref

    def launch(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Replay the captured decode on ``stream`` (default: the plan's stream, else the current one)."""
        s = stream or self.stream or torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.aa_decode_plan_launch(self.handle, s.cuda_stream), "decode_plan_launch")
            ev = torch.cuda.Event()
            ev.record(s)
        self._done = ev

    def __call__(self, images: Optional[torch.Tensor] = None):
        s = self.stream or torch.cuda.current_stream(self.device)
        if images is not None:
            if tuple(images.shape) != tuple(self.images.shape) or images.dtype != torch.float32:
                raise ValueError(f"DecodePlan: images must be {tuple(self.images.shape)} float32, got "
                                 f"{tuple(images.shape)} {images.dtype}")
            with torch.cuda.device(self.device), torch.cuda.stream(s):
                self.images.copy_(images, non_blocking=True)
        self.launch(s)
        return self.ids, self.alpha, self.beta

    def close(self) -> None:
        """Destroy the graph once its last replay has completed (waits for that replay only)."""
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            if self._done is not None:
                self._done.synchronize()
            self.lib.aa_decode_plan_destroy(h)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Encoder2Decoder(nn.Module):
    """adaptive_attention.Encoder2Decoder on MI355X kernels."""

    _captures = 0  # decode plans captured in this process (DecodePlan; sampler itself never captures)

    def __init__(self, cf, trunk: bool = False):
        """``trunk=True`` adds the ResNet-152 trunk (``encoder.resnet_conv``, keys as the
        reference's torchvision module): ``sampler`` / ``beam_search`` / ``forward`` then take images
        [B,3,224,224]; otherwise they take post-trunk features [B,2048,7,7]."""
        nn.Module.__init__(self)
        E, H, V = cf.adaptive_word_embed_size, cf.adaptive_lstm_hidden_size, cf.vocab_length
        self.encoder = AttentiveCNN(E, H, cf, trunk=trunk)
        self.has_trunk = bool(trunk)
        self.trunk_fold = True  # eval-mode trunk runs with BatchNorm folded into the convolutions
        self._folded = None
        self.decoder = Decoder(E, V, H, cf)
        object.__setattr__(self.encoder, "_owner", self)
        object.__setattr__(self.decoder, "_owner", self)
        self.dims = Dims(embed=E, hidden=H, vocab=V)
        self._pack_key = None
        self._packed = None
        self._model = None
        self.fp32_encoder = False  # True: V GEMM on fp32 MFMA instead of the fp32-accurate bf16x3 split
        # True: teacher-forced training (forward()) with every GEMM on bf16 MFMA (bf16 operands, fp32
        # accumulation: BASELINE config 5); False: fp32 GEMMs
        self.train_bf16 = False
        # True: sampler() shards the batch over the ranks of the default torch.distributed group
        # (one process per GPU) and all-gathers the results (sharded_sampler); opt-in
        self.distributed_sampler = False
        # sampler() over several GPUs of this process (the reference's sampler wraps the encoder in
        # nn.DataParallel whenever torch.cuda.device_count() > 1, adaptive_attention.py:178-181):
        # None = as the reference (every visible device when there is more than one, unless a
        # multi-rank process group is initialised); False = this device only; True = every visible
        # device; or a list of device indices (the first should be the images' device).
        # single-process multi-device sampler (device_parallel.py): opt-in -- True (every visible
        # device) or a device list; False / None keep the decode on the images' device
        self.device_parallel = False
        # the encoder's a_g branch on a second stream (aa_greedy_decode_aux): off, measured slower
        self.decode_aux_stream = False
        self._replicas = {}  # device index -> device_parallel._Replica

    # ---- weights -------------------------------------------------------------------------------
    def load_synthetic(self, seed: int = 123, bias_noise: float = 0.0) -> "Encoder2Decoder":
        """Load the counter-based synthetic weights (adaptive_amd.synth) — identical on every host."""
        from .synth import make_weights
        sd = make_weights(seed, self.dims, bias_noise=bias_noise)
        dev = next(self.parameters()).device
        full = {k: torch.from_numpy(v).to(dev) for k, v in sd.items()}
        if self.has_trunk:  # the trunk keeps its own (torchvision-style random) initialisation
            full.update({"encoder.resnet_conv." + k: v for k, v in self.encoder.resnet_conv.state_dict().items()})
        self.load_state_dict(full, strict=True)
        return self

    def load_state_dict(self, state_dict, strict: bool = True, **kw):
        # a real checkpoint (train.py:177) also carries the ResNet trunk under encoder.resnet_conv.*:
        # kept when this model has the trunk, dropped when it runs on post-trunk features.
        if self.has_trunk:
            sd = dict(state_dict)
        else:
            sd = {k: v for k, v in state_dict.items() if not k.startswith("encoder.resnet_conv.")}
        self._folded = None
        return super().load_state_dict(sd, strict=strict, **kw)

    # ---- trunk (baseline_attention.py:43) -------------------------------------------------------
    def _trunk_key(self):
        return tuple((t.data_ptr(), t._version) for t in self.encoder.resnet_conv.state_dict().values())

    def features(self, images: torch.Tensor) -> torch.Tensor:
        """Post-trunk features A [B,2048,7,7] for images [B,3,H,W] (``resnet_conv(images)``,
        baseline_attention.py:43) — PyTorch-ROCm convolutions (MIOpen); in eval mode without
        autograd (sampler, beam_search) with the BatchNorms folded into the convolutions (cached
        until a trunk tensor changes).  Without a
        trunk, ``images`` must already be post-trunk features and are returned as they are."""
        if not self.has_trunk or (images.dim() == 4 and images.size(1) == self.dims.channels):
            return images
        if images.dim() != 4 or images.size(1) != 3:
            raise ValueError(f"images must be [B,3,H,W] (or post-trunk [B,{self.dims.channels},7,7]), got {tuple(images.shape)}")
        if not images.is_cuda:
            raise RuntimeError("adaptive_amd: images must be a CUDA (ROCm) tensor")
        trunk = self.encoder.resnet_conv
        if self.training or not self.trunk_fold or torch.is_grad_enabled():
            A = trunk(images)  # train-mode BN, or gradients wanted: the module itself
        else:
            key = self._trunk_key()
            if self._folded is None or self._folded[0] != key:
                from .trunk import fold_bn
                self._folded = (key, fold_bn(trunk))
            with torch.no_grad():
                A = self._folded[1](images.contiguous(memory_format=torch.channels_last))
        if tuple(A.shape[1:]) != (self.dims.channels, 7, 7):
            raise ValueError(f"trunk output {tuple(A.shape)} is not [B,{self.dims.channels},7,7] (images must be 224x224)")
        return A.contiguous()

    def zero_grad(self, set_to_none: bool = True) -> None:
        """nn.Module.zero_grad (train.py:203) with its set_to_none=True path as one walk over the
        modules' parameter dicts (every parameter of every submodule, each once) instead of
        parameters()'s generator chain -- the same parameters, ≈ 0.07 ms less host time per training
        step; set_to_none=False is nn.Module's own."""
        if not set_to_none or getattr(self, "_is_replica", False):
            return super().zero_grad(set_to_none)
        stack, seen = [self], set()
        while stack:
            m = stack.pop()
            for q in m._parameters.values():
                if q is not None and q.grad is not None and id(q) not in seen:
                    seen.add(id(q))
                    q.grad = None
            stack.extend(c for c in m._modules.values() if c is not None)

    def _ref_params(self) -> list:
        """The 21 reference parameters in aa_ref_weights order, looked up through the modules'
        parameter dicts on every call (so a replaced Parameter is seen) -- a few dict lookups per
        parameter instead of named_parameters()'s walk over every module (≈0.07 ms per training step)."""
        out = []
        for mods, name in _WEIGHT_PATHS:
            m = self
            for a in mods:
                m = m._modules[a]
            out.append(m._parameters[name])
        return out

    def _c_dims(self) -> _lib.Dims:
        d = self.dims
        return _lib.Dims(d.embed, d.hidden, d.vocab, d.channels, d.spatial)

    def _model_struct(self) -> _lib.Model:
        """Pack parameters if any changed since the last pack (data_ptr + version counters)."""
        params = dict(self.named_parameters())
        names = [k for _, k in _lib.WEIGHT_FIELDS]
        dev = params[names[0]].device
        if dev.type != "cuda":
            raise RuntimeError("adaptive_amd.Encoder2Decoder runs on the GPU only: call .cuda() first")
        key = tuple((params[n].data_ptr(), params[n]._version) for n in names)
        if key == self._pack_key and self._model is not None:
            return self._model
        lib = _lib.load()
        cd = self._c_dims()
        _lib.check(lib.aa_check_dims(cd), "dims")
        nbytes = lib.aa_packed_bytes(cd)
        for n in names:
            p = params[n]
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                raise RuntimeError(f"adaptive_amd: parameter {n} must be contiguous fp32 on {dev}")
        packed = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        model = _lib.Model(cd, packed.data_ptr(), nbytes)
        w = _lib.RefWeights(**{f: params[k].data_ptr() for f, k in _lib.WEIGHT_FIELDS})
        with torch.cuda.device(dev):
            _lib.check(lib.aa_pack_weights(model, w, _lib.stream_handle()), "pack_weights")
        self._packed, self._model, self._pack_key = packed, model, key
        return model

    def _check_images(self, images: torch.Tensor) -> torch.Tensor:
        d = self.dims
        if images.dim() != 4 or tuple(images.shape[1:]) != (d.channels, 7, 7):
            raise ValueError(f"images must be post-trunk features [B,{d.channels},7,7], got {tuple(images.shape)}")
        if not images.is_cuda:
            raise RuntimeError("adaptive_amd: images must be a CUDA (ROCm) tensor")
        if images.dtype != torch.float32:
            raise TypeError("adaptive_amd: images must be float32")
        return images.contiguous()

    # ---- Encoder2Decoder.sampler (adaptive_attention.py:168-216) --------------------------------
    @torch.no_grad()
    def sampler(self, images: torch.Tensor, max_len: int = 30, trace: Optional[_lib.Trace] = None,
                exact_vocab: bool = False):
        """Greedy decode -> (ids [B,max_len] int64, alpha [B,max_len,49], beta [B,max_len,1]).

        ``exact_vocab=True`` computes every fp32 logit; the default screens with bf16 under a rigorous
        error bound and rescores the candidates in exact fp32 -- the ids are identical.  Every call
        launches the kernels directly on the current stream (about 4 max_len + 6 launches from one
        C call); nothing is cached per input buffer and no caller tensor is retained after the call,
        so a fresh batch per call (code_src/tools/utils.py:167-171) costs what a resident one does.
        For repeated decodes of one shape, ``DecodePlan`` replays a captured hipGraph over its own
        buffers.
        Several GPUs in this process (``self.device_parallel = True`` or a device list; opt-in, the
        counterpart of the reference's ``torch.cuda.device_count() > 1`` test,
        adaptive_attention.py:178-181): the rows are split into contiguous blocks, one per device,
        decoded concurrently (device_parallel.py) and gathered onto the images' device -- the same
        values as one decode of all rows.
        With ``self.distributed_sampler = True`` and an initialised multi-rank process group, every
        rank passes the whole batch and the call runs ``sharded_sampler`` (one process per GPU)."""
        if trace is None:
            import torch.distributed as dist
            multi_rank = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
            if self.distributed_sampler and multi_rank:
                return self.sharded_sampler(images, max_len, exact_vocab=exact_vocab)
            devices = self._parallel_devices(images, multi_rank)
            if devices is not None:
                from .device_parallel import parallel_sampler
                return parallel_sampler(self, images, int(max_len), devices, exact_vocab=exact_vocab)
        return self._sampler_local(images, max_len, trace, exact_vocab)

    def _parallel_devices(self, images: torch.Tensor, multi_rank: bool):
        """Device indices for a single-process multi-device decode, or None (this device only)."""
        mode = self.device_parallel
        if mode is False or mode is None or not images.is_cuda:  # opt-in (see __init__)
            return None
        home = images.device.index if images.device.index is not None else torch.cuda.current_device()
        if mode is True:
            devs = [home] + [d for d in range(torch.cuda.device_count()) if d != home]
        else:
            devs = [int(d) for d in mode]
        return devs if len(devs) > 1 else None

    @torch.no_grad()
    def _sampler_local(self, images, max_len, trace=None, exact_vocab=False):
        images = self._check_images(self.features(images))
        B, T, dev = images.size(0), int(max_len), images.device
        ids = torch.empty(B, T, dtype=torch.int64, device=dev)
        alpha = torch.empty(B, T, ATT, dtype=torch.float32, device=dev)
        beta = torch.empty(B, T, 1, dtype=torch.float32, device=dev)
        self._decode_into(images, T, ids, alpha, beta, trace=trace, exact_vocab=exact_vocab)
        return ids, alpha, beta

    def _decode_into(self, images, T, ids, alpha, beta, trace=None, exact_vocab=False, stream=None):
        """aa_greedy_decode_aux of ``images`` [B,C,7,7] (checked, on the model's device) into the
        given contiguous outputs, on ``stream`` (default: the current stream)."""
        model = self._model_struct()
        lib = _lib.load()
        B, dev = images.size(0), images.device
        flags = (_lib.DECODE_EXACT_VOCAB if exact_vocab else 0) | self._decode_flags()
        ws = self._workspace(lib.aa_decode_workspace_bytes(self._c_dims(), B, T), dev)
        with torch.cuda.device(dev):
            s = stream or torch.cuda.current_stream(dev)
            # one stream by default: the encoder's a_g branch (heads, x_g) beside the VWv GEMM on a
            # second stream measured slower than the whole decode on one stream (the cross-queue event
            # waits cost more than the overlap saves: 442 vs 448-457 K captions/s, A/B)
            aux = None
            if self.decode_aux_stream:
                aux = self._aux_stream(dev)
                aux.wait_stream(s)  # (the library forks/joins through events too)
            rc = lib.aa_greedy_decode_aux(model, images.data_ptr(), B, T, ids.data_ptr(), alpha.data_ptr(),
                                          beta.data_ptr(), _lib.ptr(ws), ws.numel() if ws is not None else 0,
                                          trace, flags, s.cuda_stream, aux.cuda_stream if aux is not None else None)
        _lib.check(rc, "greedy_decode")

    @torch.no_grad()
    def sharded_sampler(self, images: torch.Tensor, max_len: int = 30, total: Optional[int] = None, group=None,
                        gather_attention: bool = True, exact_vocab: bool = False):
        """Multi-rank ``sampler``: the one-process-per-GPU counterpart of the reference's
        self-distributing sampler (``nn.DataParallel`` over every visible GPU,
        adaptive_attention.py:178-181).  Every rank of ``group`` (``torch.distributed``; ``nccl`` =
        RCCL on ROCm) calls it; rank r decodes the contiguous row block ``shard_bounds(total,
        world, r)`` and one all-gather of the ids (and, with ``gather_attention``, alpha / beta)
        returns the whole batch's results on every rank -- the same values as one ``sampler`` call
        over all rows (rows never interact, and no kernel's per-row arithmetic depends on the batch
        size).  ``images``: the full batch on every rank (``total=None``), or this rank's block of a
        ``total``-row batch.  ``exact_vocab`` applies to each rank's local decode as in ``sampler``."""
        import torch.distributed as dist
        from . import distributed as D
        if not dist.is_initialized():
            raise RuntimeError("sharded_sampler needs an initialised torch.distributed process group")
        if total is None:
            total = images.size(0)
            images = D.local_rows(images, group)
        def local(x, t):
            return self._sampler_local(x, t, exact_vocab=exact_vocab)

        ids, alpha, beta = D.sharded_sampler(local, images, int(total), int(max_len),
                                             group=group, gather_attention=gather_attention)
        return ids, alpha, beta

    @torch.no_grad()
    def beam_search(self, images: torch.Tensor, max_len: int = 20, beam_size: int = 3, end_id: int = 2,
                    exact_vocab: Optional[bool] = None, fast: bool = False, vocab_events=None):
        """Beam-search decode (BASELINE config 4; not in the reference, semantics in
        include/adaptive_amd.h and DESIGN.md) -> (ids [B,T], alpha [B,T,49], beta [B,T,1],
        seqs [B,K,T], scores [B,K]): ids / alpha / beta of the best final beam, then every final
        beam best first with its cumulative log-probability.  ``end_id`` = the vocabulary's
        ``<end>`` (2 in build_vocab.py's order); a beam that emits it is finished; -1 disables.
        Logits are exact fp32 (the fp32 MFMA GEMM's fma chains, as the greedy path's exact mode) by
        default, in one fused launch per step (k_vexact); ``exact_vocab=True`` runs the same arithmetic
        as two launches (the plain fp32 GEMM k_vocab, then k_gsumm) -- the cross-check, bitwise equal;
        ``fast=True`` (or ``exact_vocab=False``) computes the logits by bf16x3 MFMA with fused
        log-sum-exp summaries -- fp32-accurate but not bitwise, so a near-tie between two candidates
        can be decided differently (opt-in speed mode).  ``vocab_events``: address of 2 * max_len raw
        hipEvent handles (adaptive_amd.hip_events.EventArray.ptr) recorded around each step's vocab
        stage, for per-launch timing."""
        check = False
        if exact_vocab is not None:
            if exact_vocab and fast:
                raise ValueError("exact_vocab=True contradicts fast=True")
            fast, check = not exact_vocab, bool(exact_vocab)
        images = self._check_images(self.features(images))
        model = self._model_struct()
        lib = _lib.load()
        B, T, K, dev = images.size(0), int(max_len), int(beam_size), images.device
        if not 1 <= K <= _lib.MAX_BEAM:
            raise ValueError(f"beam_size must be in [1, {_lib.MAX_BEAM}], got {K}")
        ids = torch.empty(B, T, dtype=torch.int64, device=dev)
        alpha = torch.empty(B, T, ATT, dtype=torch.float32, device=dev)
        beta = torch.empty(B, T, 1, dtype=torch.float32, device=dev)
        seqs = torch.empty(B, K, T, dtype=torch.int64, device=dev)
        scores = torch.empty(B, K, dtype=torch.float32, device=dev)
        nbytes = lib.aa_beam_workspace_bytes(self._c_dims(), B, T, K)
        if nbytes == 0 and B > 0 and T > 0:
            raise ValueError(f"unsupported beam configuration B={B} T={T} K={K} for {self.dims}")
        ws = self._workspace(nbytes, dev)
        with torch.cuda.device(dev):
            rc = lib.aa_beam_decode(model, images.data_ptr(), B, T, K, int(end_id), ids.data_ptr(), seqs.data_ptr(),
                                    scores.data_ptr(), alpha.data_ptr(), beta.data_ptr(), _lib.ptr(ws),
                                    ws.numel() if ws is not None else 0,
                                    (_lib.BEAM_FAST if fast else 0) | (_lib.DECODE_EXACT_VOCAB if check else 0),
                                    _lib.stream_handle(),
                                    vocab_events)
        _lib.check(rc, "beam_decode")
        return ids, alpha, beta, seqs, scores

    def _aux_stream(self, dev) -> torch.cuda.Stream:
        """The side stream of ``aa_greedy_decode_aux`` on ``dev``: the process's "decode-aux" role
        stream (hip_events.role_stream: a fresh HIP stream on its own hardware queue, shared by every
        model, so building models in a loop creates no further streams)."""
        from .hip_events import role_stream
        return role_stream(dev, "decode-aux")

    def _train_aux(self, dev):
        """The second stream of aa_train_forward_aux / aa_train_backward_aux (the weight gradients and
        the encoder's V GEMM beside the LSTM recurrence; bit-identical to one stream): the process's
        "train-aux" role stream, or None (one stream) when ``train_aux_stream`` is False."""
        if not getattr(self, "train_aux_stream", True):
            return None
        from .hip_events import role_stream
        return role_stream(dev, "train-aux").cuda_stream

    def _train_flags(self) -> int:
        return _lib.TRAIN_BF16 if getattr(self, "train_bf16", False) else 0

    def _decode_flags(self) -> int:
        """Flags of a default greedy decode (what sampler passes without exact_vocab), plus
        ``decode_extra_flags`` (e.g. ``_lib.DECODE_SPLIT_RESCORE``, the cross-check launch structure)."""
        return (_lib.DECODE_FP32_ENCODER if self.fp32_encoder else 0) | int(getattr(self, "decode_extra_flags", 0))

    def _workspace(self, nbytes: int, dev) -> Optional[torch.Tensor]:
        if nbytes == 0:
            return None
        ws = getattr(self, "_ws", None)
        if ws is None or ws.numel() < nbytes or ws.device != dev:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            self._ws = ws
        return ws

    # ---- AttentiveCNN.forward (baseline_attention.py:36-62) -------------------------------------
    @torch.no_grad()
    def _encode(self, images: torch.Tensor):
        images = self._check_images(self.features(images))
        model = self._model_struct()
        lib = _lib.load()
        d, B, dev = self.dims, images.size(0), images.device
        a_g = torch.empty(B, d.channels, device=dev)
        V = torch.empty(B, ATT, d.hidden, device=dev)
        v_g = torch.empty(B, d.embed, device=dev)
        h0 = torch.empty(B, 1, d.hidden, device=dev)
        c0 = torch.empty(B, 1, d.hidden, device=dev)
        VWv = torch.empty(B, ATT, 64, device=dev)
        with torch.cuda.device(dev):
            rc = lib.aa_encoder_tail(model, images.data_ptr(), B, a_g.data_ptr(), V.data_ptr(), v_g.data_ptr(),
                                     h0.data_ptr(), c0.data_ptr(), VWv.data_ptr(),
                                     _lib.DECODE_FP32_ENCODER if self.fp32_encoder else 0, _lib.stream_handle())
        _lib.check(rc, "encoder_tail")
        return V, v_g, (h0, c0), a_g, VWv

    # ---- Decoder.forward (baseline_attention.py:148-194) ------------------------------------------
    @torch.no_grad()
    def _decode_step(self, V, v_g, captions, states):
        """One-token captions [B,1]: the sampling step (aa_decode_step, sentinel h_{t-1} = 0).
        Whole captions [B,T], T > 1: the teacher-forced recurrence over T steps (aa_decoder_forward,
        the forward kernels of the training path) -> scores [B,T,V], alpha [B,T,49], beta [B,T,1],
        (h, c) [1,B,H] after the last step.  No autograd graph here: gradients flow through
        ``Encoder2Decoder.forward`` (aa_train_forward / aa_train_backward)."""
        d = self.dims
        if captions.dim() != 2:
            raise ValueError(f"captions must be [B, T] token ids, got {tuple(captions.shape)}")
        B, dev = V.size(0), V.device
        if states is None:
            raise ValueError("states (h, c) are required")
        if captions.size(1) != 1:
            return self._decode_steps(V, v_g, captions, states)
        h, c = states
        # accept [1,B,H] (LSTM layout) or [B,1,H] (encoder output layout)
        h = h.reshape(B, d.hidden).contiguous()
        c = c.reshape(B, d.hidden).contiguous()
        tokens = captions.reshape(B).to(torch.int64).contiguous()
        if B and (int(tokens.min()) < 0 or int(tokens.max()) >= d.vocab):
            raise IndexError("index out of range in self (embedding)")  # nn.Embedding's error
        model = self._model_struct()
        lib = _lib.load()
        V = V.contiguous()
        v_g = v_g.contiguous()
        h_out = torch.empty(1, B, d.hidden, device=dev)
        c_out = torch.empty(1, B, d.hidden, device=dev)
        scores = torch.empty(B, 1, d.vocab, device=dev)
        tok_out = torch.empty(B, dtype=torch.int64, device=dev)
        alpha = torch.empty(B, 1, ATT, device=dev)
        beta = torch.empty(B, 1, 1, device=dev)
        ws = self._workspace(lib.aa_step_workspace_bytes(self._c_dims(), B), dev)
        with torch.cuda.device(dev):
            rc = lib.aa_decode_step(model, B, tokens.data_ptr(), V.data_ptr(), None, v_g.data_ptr(), h.data_ptr(),
                                    c.data_ptr(), h_out.data_ptr(), c_out.data_ptr(), scores.data_ptr(),
                                    tok_out.data_ptr(), alpha.data_ptr(), beta.data_ptr(), _lib.ptr(ws),
                                    ws.numel() if ws is not None else 0, _lib.stream_handle())
        _lib.check(rc, "decode_step")
        self._last_tokens = tok_out
        return scores, alpha, beta, (h_out, c_out)

    def _decode_steps(self, V, v_g, captions, states):
        d = self.dims
        B, T, dev = V.size(0), captions.size(1), V.device
        if captions.size(0) != B or tuple(V.shape[1:]) != (ATT, d.hidden) or tuple(v_g.shape) != (B, d.embed):
            raise ValueError("decoder: V [B,49,H], v_g [B,E] and captions [B,T] must agree")
        h, c = states
        h = h.reshape(B, d.hidden).float().contiguous()
        c = c.reshape(B, d.hidden).float().contiguous()
        caps = captions.to(device=dev, dtype=torch.int64).contiguous()
        if B and (int(caps.min()) < 0 or int(caps.max()) >= d.vocab):
            raise IndexError("index out of range in self (embedding)")  # nn.Embedding's error
        for x in (V, v_g, h, c):
            if not x.is_cuda:
                raise RuntimeError("adaptive_amd: decoder inputs must be CUDA (ROCm) tensors")
        lib = _lib.load()
        params = dict(self.named_parameters())
        w = _lib.RefWeights(**{f: params[k].data_ptr() for f, k in _lib.WEIGHT_FIELDS})
        V, v_g = V.float().contiguous(), v_g.float().contiguous()
        scores = torch.empty(B, T, d.vocab, device=dev)
        alpha = torch.empty(B, T, ATT, device=dev)
        beta = torch.empty(B, T, 1, device=dev)
        h_out = torch.empty(1, B, d.hidden, device=dev)
        c_out = torch.empty(1, B, d.hidden, device=dev)
        nbytes = lib.aa_decoder_workspace_bytes(self._c_dims(), B, T)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            rc = lib.aa_decoder_forward(w, self._c_dims(), V.data_ptr(), v_g.data_ptr(), h.data_ptr(), c.data_ptr(), B,
                                        T, caps.data_ptr(), caps.stride(0), scores.data_ptr(), alpha.data_ptr(),
                                        beta.data_ptr(), h_out.data_ptr(), c_out.data_ptr(), ws.data_ptr(), nbytes,
                                        self._train_flags(), _lib.stream_handle())
        _lib.check(rc, "decoder_forward")
        return scores, alpha, beta, (h_out, c_out)

    # ---- AdaptiveBlock.mlp on given rows (adaptive_attention.py:132) ----------------------------
    @torch.no_grad()
    def vocab_logits(self, u: torch.Tensor, cols: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Exact fp32 logits u W_m^T + b_m for u [B,H] (CUDA); all columns, or only ``cols`` [B,n]
        (int32/int64, rescoring in the same fma order, so bit-identical to the full logits)."""
        model = self._model_struct()
        lib = _lib.load()
        u = u.contiguous().float()
        B = u.size(0)
        with torch.cuda.device(u.device):
            if cols is None:
                out = torch.empty(B, self.dims.vocab, device=u.device)
                rc = lib.aa_vocab_logits(model, B, u.data_ptr(), out.data_ptr(), _lib.stream_handle())
            else:
                cols = cols.to(device=u.device, dtype=torch.int32).contiguous()
                out = torch.empty(B, cols.size(1), device=u.device)
                rc = lib.aa_vocab_logits_at(model, B, u.data_ptr(), cols.data_ptr(), cols.size(1), out.data_ptr(),
                                            _lib.stream_handle())
        _lib.check(rc, "vocab_logits")
        return out

    # ---- Encoder2Decoder.forward (baseline_attention.py:206-230): teacher-forced training ------
    def forward(self, images, captions, lengths):
        """Teacher-forced forward -> ``PackedSequence`` of the scores, exactly as the reference's
        ``pack_padded_sequence(scores, lengths, batch_first=True)``; differentiable w.r.t. every
        parameter (HIP forward and backward kernels, C-ABI ``aa_train_*``), so train.py's closure
        (CrossEntropyLoss on ``packed[0]``, ``loss.backward()``, clip_grad_norm_, optimizer.step)
        runs unchanged.  ``images`` are post-trunk features [B,2048,7,7], or images [B,3,224,224]
        when the model has the trunk (its forward and backward then run in PyTorch-ROCm and the
        HIP backward hands it dL/dA, so CNN fine-tuning, train.py:89, works unchanged)."""
        from torch.nn.utils.rnn import PackedSequence
        images = self._check_images(self.features(images))
        lengths = tuple(map(int, lengths.tolist() if torch.is_tensor(lengths) else lengths))
        B = images.size(0)
        if captions.dim() != 2 or captions.size(0) != B or len(lengths) != B:
            raise ValueError("captions must be [B, L] and lengths a list of B ints")
        dev = images.device
        # per distinct lengths list, validated once and cached: the lengths on the device (a fresh
        # torch.tensor(..., device=dev) is a pageable host->device copy, which HIP may stage
        # synchronously: the host then waits before it can queue the rest of the step) and the
        # PackedSequence batch sizes (an O(B T) Python loop, ~0.1 ms of host time per step at B = 128)
        cache = self.__dict__.setdefault("_len_dev_cache", {})
        key = (dev, lengths)
        hit = cache.get(key)
        if hit is None:
            bs = packed_batch_sizes(lengths)
            if len(cache) > 64:
                cache.clear()
            hit = cache[key] = (torch.tensor(lengths, dtype=torch.int32, device=dev),
                                torch.tensor(bs, dtype=torch.int64), sum(lengths))
        len_dev, batch_sizes, N = hit
        T = lengths[0]
        if T > captions.size(1):
            raise ValueError("lengths exceed the caption width")
        caps = captions.to(device=dev, dtype=torch.int64).contiguous()
        data = _TeacherForced.apply(self, images, caps, len_dev, N, T, *self._ref_params())
        return PackedSequence(data, batch_sizes.clone())


def packed_batch_sizes(lengths) -> list:
    """pack_padded_sequence's ``batch_sizes`` for sorted ``lengths`` (step t: the rows longer than t),
    in O(B + T); raises ValueError, as the reference's packing would, for lengths that are not
    positive and sorted in decreasing order."""
    B = len(lengths)
    if B == 0 or any(n < 1 for n in lengths) or any(lengths[i] < lengths[i + 1] for i in range(B - 1)):
        raise ValueError("lengths must be positive and sorted in decreasing order (pack_padded_sequence)")
    bs = [0] * lengths[0]
    for n in lengths:
        bs[n - 1] += 1
    for t in range(lengths[0] - 2, -1, -1):
        bs[t] += bs[t + 1]
    return bs


_WEIGHT_PATHS = [(tuple(k.split(".")[:-1]), k.split(".")[-1]) for _, k in _lib.WEIGHT_FIELDS]


class _TeacherForced(torch.autograd.Function):
    """HIP teacher-forced forward / backward (aa_train_forward / aa_train_backward).  The workspace
    of the forward call carries the activations to the backward call."""

    @staticmethod
    def forward(ctx, owner, images, caps, len_dev, N, T, *params):
        lib = _lib.load()
        d = owner._c_dims()
        B = images.size(0)
        nbytes = lib.aa_train_workspace_bytes(d, B, T)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=images.device)
        scores = torch.empty(N, owner.dims.vocab, device=images.device)
        w = _lib.RefWeights(*[p.data_ptr() for p in params])
        with _lib.on_device(images.device):
            rc = lib.aa_train_forward_aux(w, d, images.data_ptr(), B, T, caps.data_ptr(), caps.stride(0),
                                          len_dev.data_ptr(), scores.data_ptr(), N, ws.data_ptr(), nbytes,
                                          owner._train_flags(), _lib.stream_handle(), owner._train_aux(images.device))
        _lib.check(rc, "train_forward")
        ctx.owner, ctx.ws, ctx.N, ctx.T, ctx.flags = owner, ws, N, T, owner._train_flags()
        ctx.save_for_backward(images, caps, len_dev, *params)
        return scores

    @staticmethod
    def backward(ctx, dscores):
        lib = _lib.load()
        images, caps, len_dev, *params = ctx.saved_tensors
        owner = ctx.owner
        B = images.size(0)
        dscores = dscores.contiguous().float()
        grads = [torch.empty_like(p) for p in params]
        dfeats = torch.empty_like(images) if ctx.needs_input_grad[1] else None
        w = _lib.RefWeights(*[p.data_ptr() for p in params])
        g = _lib.RefWeights(*[t.data_ptr() for t in grads])
        with _lib.on_device(images.device):
            rc = lib.aa_train_backward_aux(w, owner._c_dims(), images.data_ptr(), B, ctx.T, caps.data_ptr(),
                                           caps.stride(0), len_dev.data_ptr(), dscores.data_ptr(), ctx.N, g,
                                           _lib.ptr(dfeats), ctx.ws.data_ptr(), ctx.ws.numel(), ctx.flags,
                                           _lib.stream_handle(), owner._train_aux(images.device))
        _lib.check(rc, "train_backward")
        ctx.ws = None
        return (None, dfeats, None, None, None, None, *grads)


def synthetic_features(B: int, device, seed: int = 0, row0: int = 0, dims: Dims = Dims()) -> torch.Tensor:
    """[B, C, 7, 7] U[0,1) features generated ON the GPU by aa_synth_uniform (same bits as
    adaptive_amd.synth.make_features)."""
    from .synth import stream_key
    lib = _lib.load()
    per_row = dims.channels * dims.spatial
    out = torch.empty(B, dims.channels, 7, 7, dtype=torch.float32, device=device)
    with torch.cuda.device(out.device):
        _lib.check(lib.aa_synth_uniform(out.data_ptr(), B * per_row, stream_key(seed, "features"), row0 * per_row,
                                        0.0, 1.0, _lib.stream_handle()), "synth_uniform")
    return out

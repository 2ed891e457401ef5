"""Pipelined greedy decode over a stream of batches — the reference's evaluation loop
(``coco_eval``: ``for images in data_loader: model.sampler(images)``, code_src/tools/utils.py:167-171)
with up to ``depth`` batches in flight on their own HIP streams.

One B = 512 decode is latency-bound on MI355X: its step kernels hold one or two workgroups per CU,
and the encoder GEMM cannot start before the previous batch's last step.  Batches are independent,
so batch i + 1 (encoder and first steps) runs on a second stream while batch i finishes: same
kernels, same per-batch work and the same ids bit for bit (tests/test_gpu_parity.py), more of the
chip busy.  Each slot owns its stream, workspace and output buffers; the caller's stream waits for a
batch's completion event only when that batch's result is handed out.
"""
from __future__ import annotations

import collections
from typing import Iterable, Iterator, Tuple

import torch

from . import _lib
from .adaptive_attention import ATT


class _Slot:
    def __init__(self, dev, stream):
        self.stream = stream
        self.dev = dev
        self.ws = None


class Retired(tuple):
    """One retired batch: unpacks as ``(ids, alpha, beta)``; ``.done`` is the batch's completion
    event (recorded on its slot stream, after its ids host copy) and ``.ids_host`` the pinned host
    tensor its ids were copied into (None without ``ids_host``).  The host tensor may be read only
    after ``.done`` has completed -- ``done.synchronize()``, or a synchronisation of the caller's
    stream, which ``retire`` made wait on it."""

    def __new__(cls, out, done, ids_host):
        r = super().__new__(cls, out)
        r.done, r.ids_host = done, ids_host
        return r


class DecodePipeline:
    """``for ids, alpha, beta in DecodePipeline(model, max_len=20).run(batches): ...`` — results
    in submission order, each exactly ``model.sampler(images, max_len)``'s.

    Each batch's kernels are launched directly into its slot's stream (one stream per slot: the
    encoder's side branch stays on the slot stream, since the other slots already fill the chip), so
    the process owns exactly ``depth`` busy streams.  HIP multiplexes a process's streams onto a few
    hardware queues (GPU_MAX_HW_QUEUES, 4 by default), and two slots that land on one queue
    serialise.  (Slots replaying captured decode plans measured slower, DESIGN.md §4, and were
    removed.)

    With ``raw_streams=True`` (default) the first slot runs on the model's decode side stream (the
    "decode-aux" role stream, idle while the pipeline runs: slots launch without a side stream) and the
    others on the first ``depth - 1`` of the process-wide list of fresh HIP streams
    (``hip_events.raw_streams``).  HIP hands a process's streams out round-robin over
    GPU_MAX_HW_QUEUES (4) hardware queues, and the caller's stream and the decode side stream already
    hold two: reusing the side stream keeps three slots on three distinct queues besides the caller's
    (measured, depth 3, one box: 549 K captions/s against 444 K with three fresh streams, one of which
    shared a queue).  Two pipelines alive on one device share those streams and therefore serialise
    against each other (results stay correct; only their overlap is lost).  For the same reason a
    ``sampler()`` call on the same device while pipeline batches are in flight queues its encoder side
    branch behind slot 0's whole decode and its stream then waits for it: the two serialise.  Results
    stay correct, but do not interleave ``sampler()`` with a live pipeline where overlap matters --
    submit the batch to the pipeline instead."""

    def __init__(self, model, max_len: int = 20, depth: int = 2, raw_streams: bool = True, streams=None):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.model, self.T, self.depth = model, int(max_len), int(depth)
        self.raw_streams = bool(raw_streams)
        if streams is not None and len(streams) != self.depth:
            raise ValueError("streams: one per batch in flight")
        self._streams = streams
        self._slots = None
        self._pending = collections.deque()
        self._n = 0

    def _slot(self, dev) -> _Slot:
        if self._slots is None:
            if self._streams is not None:
                streams = list(self._streams)
            elif self.raw_streams:  # the decode side stream + fresh HIP streams: distinct hardware queues
                from .hip_events import raw_streams
                streams = [self.model._aux_stream(dev)] + raw_streams(dev, self.depth - 1)
            else:
                streams = [torch.cuda.Stream(device=dev) for _ in range(self.depth)]
            self._slots = [_Slot(dev, st) for st in streams]
        return self._slots[self._n % self.depth]

    @torch.no_grad()
    def submit(self, images: torch.Tensor, ids_host: torch.Tensor = None) -> None:
        """Queue one batch (post-trunk features, or images when the model has the trunk).
        ``ids_host``: a pinned host tensor [B, T] int64 that receives the batch's ids by a copy on the
        slot's own stream, as the batch's last operation (no work for the caller's stream)."""
        m = self.model
        if len(self._pending) >= self.depth:
            raise RuntimeError("pipeline full: retire() a result first")
        images = m._check_images(m.features(images))
        model = m._model_struct()  # (re)packs on the current stream if the weights changed
        lib = _lib.load()
        B, T, dev = images.size(0), self.T, images.device
        slot = self._slot(dev)
        ready = torch.cuda.Event()
        ready.record()  # images (and any repack) are ready on the caller's stream
        s = slot.stream
        s.wait_event(ready)
        images.record_stream(s)
        flags = m._decode_flags()  # the same flags sampler() passes (fp32_encoder included)
        with torch.cuda.device(dev), torch.cuda.stream(s):
            ids = torch.empty(B, T, dtype=torch.int64, device=dev)
            alpha = torch.empty(B, T, ATT, dtype=torch.float32, device=dev)
            beta = torch.empty(B, T, 1, dtype=torch.float32, device=dev)
            nbytes = lib.aa_decode_workspace_bytes(m._c_dims(), B, T)
            if nbytes and (slot.ws is None or slot.ws.numel() < nbytes):
                slot.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            # the other slots already fill the chip: one stream per slot (no aux stream)
            rc = lib.aa_greedy_decode_aux(model, images.data_ptr(), B, T, ids.data_ptr(), alpha.data_ptr(),
                                          beta.data_ptr(), _lib.ptr(slot.ws) if nbytes else None, nbytes, None,
                                          flags, s.cuda_stream, None)
            _lib.check(rc, "greedy_decode")
            out = (ids, alpha, beta)
            if ids_host is not None:
                ids_host.copy_(out[0], non_blocking=True)
            done = torch.cuda.Event()
            done.record(s)
        self._pending.append((done, out, images, ids_host))
        self._n += 1

    def retire(self) -> "Retired":
        """The oldest queued batch's (ids, alpha, beta) as a ``Retired`` tuple; the caller's stream
        waits for it (the host is not synchronised: read ``ids_host`` only after ``.done``)."""
        done, out, _, ids_host = self._pending.popleft()
        cur = torch.cuda.current_stream()
        cur.wait_event(done)
        for t in out:
            t.record_stream(cur)
        return Retired(out, done, ids_host)

    def run(self, batches: Iterable[torch.Tensor], ids_host=None) -> Iterator[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """``ids_host``: optional list of pinned host tensors, used round-robin per submitted batch
        (see ``submit``); a buffer is handed to a new batch only after its previous batch was
        retired when the list holds more than ``depth`` buffers.  Each yielded ``Retired`` names its
        buffer (``.ids_host``), readable once ``.done`` has completed."""
        for i, images in enumerate(batches):
            if len(self._pending) >= self.depth:
                yield self.retire()
            self.submit(images, None if ids_host is None else ids_host[i % len(ids_host)])
        while self._pending:
            yield self.retire()

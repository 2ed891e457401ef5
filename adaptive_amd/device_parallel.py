"""Single-process multi-device greedy decode: the counterpart of the reference's self-distributing
sampler, which wraps the encoder in ``nn.DataParallel`` over every visible GPU whenever
``torch.cuda.device_count() > 1`` (code_src/models/adaptive_attention.py:178-181; the per-step
decoder is data-parallel the same way, baseline_attention.py:184-187), with no launcher and no
process group -- so an unchanged ``coco_eval`` (code_src/tools/utils.py:167-171) started by an
unchanged ``main.py`` on a multi-GPU node uses every GPU.

MI355X form: captions are independent, so the batch is split into contiguous row blocks, one per
device (``plan_shards``), and each block is decoded entirely on its device with no per-step
communication:

* the home block (the images' own device) is decoded in place on the caller's stream;
* every other device holds a replica of the packed weights (``_Replica``: the 21 parameter tensors
  copied to that device once per weight version and packed there by ``aa_pack_weights``) and a
  ``DecodePlan`` per block shape -- a captured hipGraph over buffers the plan owns, so one host call
  launches the whole decode and the host thread is not the bottleneck of N devices;
* per remote device, on its "device-parallel" role stream: wait for the caller's stream, peer-copy
  the block's features into the plan's input buffer, replay the plan, peer-copy ids / alpha / beta
  back into the caller's output rows (hipMemcpyAsync on that stream only), record a completion
  event;
* the caller's stream waits for every completion event, so the results are ordered like any other
  op on it (and the caching allocator may reuse the caller's inputs only after the copies).

Every kernel's per-row arithmetic is independent of the batch size, so the gathered ids, alpha and
beta equal one decode of all rows bit for bit (``tests/test_gpu_device_parallel.py``).  Peer access
between the home device and each remote device is enabled explicitly (``hipDeviceEnablePeerAccess``,
idempotent) before the first peer copy.  The RCCL multi-process path (``adaptive_amd.distributed``)
is unchanged.

Opt-in (``model.device_parallel = True`` or a device list): this path has run only on a one-GPU
box, with the device listed repeatedly and ``FORCE_REMOTE`` set so the extra blocks take the
remote-device machinery (replica pack, ``_ReplicaView`` plans, stream-local copies) on the same
device.  It has never touched a second physical device, so a plain ``sampler`` call stays on the
images' device unless asked.
"""
from __future__ import annotations

import collections
from typing import Dict, List, Sequence, Tuple

import torch

from . import _lib
from .adaptive_attention import ATT, DecodePlan

MAX_PLANS_PER_DEVICE = 2  # block shapes kept captured per device (LRU); eviction waits for that plan only
# test hook: treat every block as remote (a weight replica packed on its device, a plan over the
# replica's weights, copies in and out) even on the images' own device -- how a one-GPU box runs the
# remote-device machinery (tests/test_gpu_device_parallel.py)
FORCE_REMOTE = False


def plan_shards(B: int, devices: Sequence[int]) -> List[Tuple[int, int, int]]:
    """Contiguous row blocks ``(device, lo, hi)`` for a B-row batch over ``devices`` (the first
    ``B % n`` blocks one row longer, as ``distributed.shard_bounds``); empty blocks are dropped.
    The first device (the images' own) takes the first block."""
    n = len(devices)
    if n < 1:
        raise ValueError("plan_shards needs at least one device")
    if B < 0:
        raise ValueError(f"bad batch size {B}")
    q, r = divmod(B, n)
    out, lo = [], 0
    for i, d in enumerate(devices):
        hi = lo + q + (1 if i < r else 0)
        if hi > lo:
            out.append((int(d), lo, hi))
        lo = hi
    return out


class _Replica:
    """The model's packed weights on another device (or, for the home device, the model's own), plus
    that device's captured decode plans keyed by (rows, max_len, flags)."""

    def __init__(self, owner, device: int):
        self.device = torch.device("cuda", device)
        self.home = None  # set by refresh(): the owner's packed weights live on this device
        self.model = None
        self.params: Dict[str, torch.Tensor] = {}
        self.packed = None
        self.plans: "collections.OrderedDict[tuple, DecodePlan]" = collections.OrderedDict()
        self._owner_key = None

    def refresh(self, owner, stream) -> None:
        """(Re)pack on this device if the owner's weights changed since the last pack."""
        owner._model_struct()
        # recomputed every call: the model may have moved to another device since this replica was made
        home = owner._packed.device == self.device and not FORCE_REMOTE
        if self._owner_key == owner._pack_key and self.home == home:
            return
        for p in self.plans.values():
            p.close()
        self.plans.clear()
        self._owner_key = owner._pack_key
        self.home = home
        if self.home:
            self.params, self.packed, self.model = {}, None, None
            return
        lib = _lib.load()
        named = dict(owner.named_parameters())
        with torch.cuda.device(self.device), torch.cuda.stream(stream):
            # wait for the owner's current stream (the parameters' last writes) before copying them
            stream.wait_stream(torch.cuda.current_stream(owner._packed.device))
            self.params = {k: named[k].detach().to(self.device, non_blocking=True) for _, k in _lib.WEIGHT_FIELDS}
            cd = owner._c_dims()
            nbytes = lib.aa_packed_bytes(cd)
            self.packed = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self.model = _lib.Model(cd, self.packed.data_ptr(), nbytes)
            w = _lib.RefWeights(**{f: self.params[k].data_ptr() for f, k in _lib.WEIGHT_FIELDS})
            _lib.check(lib.aa_pack_weights(self.model, w, stream.cuda_stream), "pack_weights (replica)")

    def plan(self, owner, rows: int, T: int, exact: bool, stream) -> DecodePlan:
        key = (rows, T, bool(exact), owner._decode_flags())
        plan = self.plans.get(key)
        if plan is None:
            plan = _ReplicaPlan(self, owner, rows, T, exact, stream) if not self.home else \
                DecodePlan(owner, rows, T, exact_vocab=exact, stream=stream)
            self.plans[key] = plan
            while len(self.plans) > MAX_PLANS_PER_DEVICE:
                self.plans.popitem(last=False)[1].close()
        self.plans.move_to_end(key)
        return plan


class _ReplicaView:
    """The attributes DecodePlan reads from a model, pointing at a replica's packed weights."""

    def __init__(self, replica: _Replica, owner):
        self._replica, self._owner = replica, owner
        self.dims = owner.dims
        self._packed = replica.packed
        self._pack_key = ("replica", replica.device.index, owner._pack_key)

    def _model_struct(self):
        return self._replica.model

    def _c_dims(self):
        return self._owner._c_dims()

    def _decode_flags(self):
        return self._owner._decode_flags()


def _ReplicaPlan(replica: _Replica, owner, rows: int, T: int, exact: bool, stream) -> DecodePlan:
    return DecodePlan(_ReplicaView(replica, owner), rows, T, exact_vocab=exact, stream=stream)


def _replica(owner, device: int) -> _Replica:
    rep = owner._replicas.get(device)
    if rep is None:
        rep = owner._replicas[device] = _Replica(owner, device)
    return rep


@torch.no_grad()
def parallel_sampler(owner, images: torch.Tensor, T: int, devices: Sequence[int], exact_vocab: bool = False):
    """``owner.sampler(images, T)`` with the rows split over ``devices`` (see the module docstring).
    Returns (ids, alpha, beta) on the images' device."""
    from .hip_events import copy_async, enable_peer_access, role_stream
    images = owner._check_images(owner.features(images))
    owner._model_struct()  # pack on the home device first (replicas copy the same parameters)
    B, home = images.size(0), images.device
    if T <= 0 or B == 0:
        return owner._sampler_local(images, T, exact_vocab=exact_vocab)
    shards = plan_shards(B, devices)
    ids = torch.empty(B, T, dtype=torch.int64, device=home)
    alpha = torch.empty(B, T, ATT, dtype=torch.float32, device=home)
    beta = torch.empty(B, T, 1, dtype=torch.float32, device=home)
    cur = torch.cuda.current_stream(home)
    ready = torch.cuda.Event()
    ready.record(cur)  # the features (and any repack) are ready on the caller's stream
    done = []
    home_shards = []
    for i, (d, lo, hi) in enumerate(shards):
        if i == 0 and d == home.index:
            home_shards.append((lo, hi))  # decoded in place after the remote launches are queued
            continue
        enable_peer_access(home.index, d)  # both directions, once per pair (no-op for d == home)
        s = role_stream(d, "device-parallel")
        rep = _replica(owner, d)
        with torch.cuda.device(d), torch.cuda.stream(s):
            s.wait_event(ready)
            rep.refresh(owner, s)
            plan = rep.plan(owner, hi - lo, T, exact_vocab, s)
            # peer copies on s alone (torch's cross-device copy_ would also block the caller's stream
            # behind this device's decode, serialising the devices)
            copy_async(plan.images, images[lo:hi], s)
            plan.launch(s)
            copy_async(ids[lo:hi], plan.ids, s)
            copy_async(alpha[lo:hi], plan.alpha, s)
            copy_async(beta[lo:hi], plan.beta, s)
            ev = torch.cuda.Event()
            ev.record(s)
            done.append(ev)
    for lo, hi in home_shards:
        owner._decode_into(images[lo:hi], T, ids[lo:hi], alpha[lo:hi], beta[lo:hi], exact_vocab=exact_vocab)
    for ev in done:
        cur.wait_event(ev)
    return ids, alpha, beta


__all__ = ["plan_shards", "parallel_sampler", "MAX_PLANS_PER_DEVICE"]

"""Raw hipEvent handles for the C-ABI's per-kernel timing hook (``aa_trace``).

torch's ``torch.cuda.Event`` creates its handle lazily on first ``record()``, so it cannot be handed
to a C call that records it itself; these are created eagerly through the HIP runtime already
loaded by torch (``libamdhip64.so.7``).
"""
from __future__ import annotations

import ctypes
import warnings
from ctypes import POINTER, c_float, c_int, c_void_p

import torch  # noqa: F401  (loads torch's HIP runtime first)

_hip = None


def hip() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        lib = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
        lib.hipEventCreate.argtypes = [POINTER(c_void_p)]
        lib.hipEventCreate.restype = c_int
        lib.hipEventCreateWithFlags.argtypes = [POINTER(c_void_p), ctypes.c_uint]
        lib.hipEventCreateWithFlags.restype = c_int
        lib.hipEventDestroy.argtypes = [c_void_p]
        lib.hipEventDestroy.restype = c_int
        lib.hipEventElapsedTime.argtypes = [POINTER(c_float), c_void_p, c_void_p]
        lib.hipEventElapsedTime.restype = c_int
        lib.hipEventSynchronize.argtypes = [c_void_p]
        lib.hipEventSynchronize.restype = c_int
        lib.hipEventRecord.argtypes = [c_void_p, c_void_p]
        lib.hipEventRecord.restype = c_int
        lib.hipStreamCreateWithFlags.argtypes = [POINTER(c_void_p), ctypes.c_uint]
        lib.hipStreamCreateWithFlags.restype = c_int
        lib.hipStreamDestroy.argtypes = [c_void_p]
        lib.hipStreamDestroy.restype = c_int
        lib.hipMemcpyAsync.argtypes = [c_void_p, c_void_p, ctypes.c_size_t, c_int, c_void_p]
        lib.hipMemcpyAsync.restype = c_int
        _hip = lib
    return _hip


# timing-only events: hipEventReleaseToDevice (a device-scope release when the event is recorded
# instead of a system-scope one: no cache writeback / invalidate between the timed kernels), else
# hipEventDisableSystemFence, else a default event -- the first flag set this HIP runtime accepts
# (hip_runtime_api.h); ``timing_flags_used()`` names it
TIMING_FLAG_CHOICES = (("hipEventReleaseToDevice", 0x40000000), ("hipEventDisableSystemFence", 0x20000000),
                       ("hipEventDefault", 0x0))
_timing_flags = None


def _create_timing_event(ev) -> int:
    global _timing_flags
    h = hip()
    if _timing_flags is not None:
        return h.hipEventCreateWithFlags(ctypes.byref(ev), _timing_flags[1])
    rc = -1
    for name, flags in TIMING_FLAG_CHOICES:
        rc = h.hipEventCreateWithFlags(ctypes.byref(ev), flags)
        if rc == 0:
            _timing_flags = (name, flags)
            break
    return rc


def timing_flags_used() -> str:
    return _timing_flags[0] if _timing_flags else "none yet"


class EventArray:
    """n raw hipEvent_t handles as a C array (pass ``.ptr`` as an ``aa_event_t*``).  ``precise``:
    timing-only events (``_create_timing_event``), the default for per-kernel timing."""

    def __init__(self, n: int, precise: bool = True):
        self.n = n
        self.arr = (c_void_p * n)()
        h = hip()
        for i in range(n):
            ev = c_void_p()
            rc = _create_timing_event(ev) if precise else h.hipEventCreate(ctypes.byref(ev))
            if rc != 0:
                raise RuntimeError(f"hipEventCreate failed: {rc}")
            self.arr[i] = ev.value

    @property
    def ptr(self) -> int:
        return ctypes.addressof(self.arr)

    def elapsed_ms(self, i: int, j: int) -> float:
        h = hip()
        h.hipEventSynchronize(self.arr[j])
        ms = c_float()
        rc = h.hipEventElapsedTime(ctypes.byref(ms), self.arr[i], self.arr[j])
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed: {rc}")
        return ms.value

    def record(self, i: int, stream) -> None:
        """Record event i on ``stream`` (a torch stream)."""
        rc = hip().hipEventRecord(self.arr[i], stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed: {rc}")

    def pair_durations_ms(self, npairs: int | None = None):
        npairs = self.n // 2 if npairs is None else npairs
        return [self.elapsed_ms(2 * k, 2 * k + 1) for k in range(npairs)]

    def close(self):
        h = hip()
        for i in range(self.n):
            if self.arr[i]:
                h.hipEventDestroy(self.arr[i])
                self.arr[i] = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_raw_streams = {}
_role_streams = {}  # (device index, role) -> stream: a bounded pool, one stream per role and device


def _create(idx: int) -> "torch.cuda.ExternalStream":
    h = c_void_p()
    with torch.cuda.device(idx):
        rc = hip().hipStreamCreateWithFlags(ctypes.byref(h), 1)  # hipStreamNonBlocking
    if rc != 0:
        raise RuntimeError(f"hipStreamCreateWithFlags failed: {rc}")
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))


def _index(device) -> int:
    dev = torch.device(device)
    return dev.index if dev.index is not None else torch.cuda.current_device()


def raw_streams(device, n: int):
    """The first ``n`` of this process's SHARED fresh non-blocking HIP streams on ``device``
    (hipStreamCreateWithFlags), as torch.cuda.ExternalStream objects.  HIP assigns each new stream a
    hardware queue round-robin (GPU_MAX_HW_QUEUES, 4 by default), so streams created back to back land
    on distinct queues -- unlike streams handed out by torch's pool, whose queues were fixed when the
    pool was made.  They live as long as the process (torch's caching allocator may still record
    events on them after their user is gone), and every caller gets the same first ``n``: two users
    of this list serialise against each other on the streams they share."""
    idx = _index(device)
    have = _raw_streams.setdefault(idx, [])
    while len(have) < n:
        have.append(_create(idx))
    return have[:n]


def role_stream(device, role: str) -> "torch.cuda.ExternalStream":
    """The process's fresh non-blocking HIP stream for ``role`` on ``device`` (created on first use,
    then shared by every caller asking for the same role: e.g. the decode's aux stream, or a
    device-parallel shard stream).  The pool is bounded by the roles in use, so building models or
    pipelines in a loop creates no further streams.  Each new role's stream takes the next hardware
    queue in HIP's round-robin; like ``raw_streams`` they live as long as the process (torch's caching
    allocator may still record events on them)."""
    key = (_index(device), str(role))
    st = _role_streams.get(key)
    if st is None:
        st = _role_streams[key] = _create(key[0])
    return st


HIP_MEMCPY_DEFAULT = 4  # hipMemcpyDefault: direction from the pointers (unified addressing)
HIP_ERROR_PEER_ACCESS_ALREADY_ENABLED = 704
_peer_state = {}  # (a, b) -> peer access enabled (True) or no P2P path (False)


def enable_peer_access(a: int, b: int) -> bool:
    """Let devices ``a`` and ``b`` read and write each other's memory (hipDeviceEnablePeerAccess in
    both directions; idempotent: "already enabled" counts as success).  Done explicitly before the
    first peer copy of a single-process multi-device decode instead of relying on a side effect of
    torch's cross-device ``.to()``.  Returns False (and warns once per pair) when
    hipDeviceCanAccessPeer reports no P2P path: the decode's ``hipMemcpyAsync(hipMemcpyDefault)``
    copies then stage through the host -- slower, still correct.  Both outcomes are cached, so the
    check runs once per pair."""
    a, b = int(a), int(b)
    if a == b:
        return True
    if (a, b) in _peer_state:
        return _peer_state[(a, b)]
    h = hip()
    h.hipDeviceCanAccessPeer.argtypes = [ctypes.POINTER(c_int), c_int, c_int]
    h.hipDeviceCanAccessPeer.restype = c_int
    h.hipDeviceEnablePeerAccess.argtypes = [c_int, ctypes.c_uint]
    h.hipDeviceEnablePeerAccess.restype = c_int
    for src, dst in ((a, b), (b, a)):
        ok = c_int(0)
        rc = h.hipDeviceCanAccessPeer(ctypes.byref(ok), src, dst)
        if rc != 0 or not ok.value:
            warnings.warn(f"adaptive_amd: device {src} cannot access device {dst} directly "
                          f"(hipDeviceCanAccessPeer rc={rc}); peer copies stage through the host")
            _peer_state[(a, b)] = _peer_state[(b, a)] = False
            return False
    for src, dst in ((a, b), (b, a)):
        with torch.cuda.device(src):
            rc = h.hipDeviceEnablePeerAccess(dst, 0)
        if rc not in (0, HIP_ERROR_PEER_ACCESS_ALREADY_ENABLED):
            raise RuntimeError(f"hipDeviceEnablePeerAccess({src} -> {dst}) failed: {rc}")
    _peer_state[(a, b)] = _peer_state[(b, a)] = True
    return True


def copy_async(dst: "torch.Tensor", src: "torch.Tensor", stream) -> None:
    """dst <- src (contiguous, same shape and dtype, on any devices) by one hipMemcpyAsync queued on
    ``stream`` and on that stream ONLY.  torch's cross-device ``copy_`` instead synchronises the
    current streams of both devices around the copy (ATen's device-to-device copy), which would
    serialise the devices of a single-process multi-device decode; the caller orders this copy with
    events instead."""
    if dst.shape != src.shape or dst.dtype != src.dtype or not (dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("copy_async: dst and src must be contiguous tensors of one shape and dtype")
    n = src.numel() * src.element_size()
    if n == 0:
        return
    rc = hip().hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), n, HIP_MEMCPY_DEFAULT, stream.cuda_stream)
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed: {rc}")

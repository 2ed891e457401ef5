"""Raw hipEvent handles for the C-ABI's per-kernel timing hook (``aa_trace``).

torch's ``torch.cuda.Event`` creates its handle lazily on first ``record()``, so it cannot be handed
to a C call that records it itself; these are created eagerly through the HIP runtime already
loaded by torch (``libamdhip64.so.7``).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_float, c_int, c_void_p

import torch  # noqa: F401  (loads torch's HIP runtime first)

_hip = None


def hip() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        lib = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
        lib.hipEventCreate.argtypes = [POINTER(c_void_p)]
        lib.hipEventCreate.restype = c_int
        lib.hipEventDestroy.argtypes = [c_void_p]
        lib.hipEventDestroy.restype = c_int
        lib.hipEventElapsedTime.argtypes = [POINTER(c_float), c_void_p, c_void_p]
        lib.hipEventElapsedTime.restype = c_int
        lib.hipEventSynchronize.argtypes = [c_void_p]
        lib.hipEventSynchronize.restype = c_int
        lib.hipStreamCreateWithFlags.argtypes = [POINTER(c_void_p), ctypes.c_uint]
        lib.hipStreamCreateWithFlags.restype = c_int
        lib.hipStreamDestroy.argtypes = [c_void_p]
        lib.hipStreamDestroy.restype = c_int
        _hip = lib
    return _hip


class EventArray:
    """n raw hipEvent_t handles as a C array (pass ``.ptr`` as an ``aa_event_t*``)."""

    def __init__(self, n: int):
        self.n = n
        self.arr = (c_void_p * n)()
        h = hip()
        for i in range(n):
            ev = c_void_p()
            rc = h.hipEventCreate(ctypes.byref(ev))
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
_owned_streams = []  # streams handed out by new_raw_stream (kept alive for the process)


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


def new_raw_stream(device) -> "torch.cuda.ExternalStream":
    """A fresh non-blocking HIP stream on ``device`` that no other caller of this module gets (it
    takes the next hardware queue in HIP's round-robin at the time of the call).  Kept alive for the
    process, as ``raw_streams``."""
    st = _create(_index(device))
    _owned_streams.append(st)
    return st

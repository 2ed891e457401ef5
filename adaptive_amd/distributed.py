"""Multi-GPU greedy decode: one process per GPU, contiguous row shards, one all-gather of ids.

Captioning is embarrassingly parallel (rows never interact: SURVEY.md §8e, and every kernel's
per-row arithmetic is independent of the shard size), so rank r decodes rows [lo_r, hi_r) of the
global batch with no per-step communication, then a single all-gather of the int64 token ids
assembles [B, T] on every rank.  This replaces the reference's per-step ``nn.DataParallel``
scatter/replicate/gather (code_src/models/baseline_attention.py:184-187,
adaptive_attention.py:178-181).  Backend ``nccl`` is RCCL on ROCm (xGMI); ``gloo`` is used by the
CPU tests.
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of rows for ``rank``; the first ``total % world`` ranks get one extra row."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError(f"bad shard request total={total} world={world} rank={rank}")
    q, r = divmod(total, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    if dist.get_backend(group) == "nccl":  # RCCL: one fused all-gather into the output buffer
        dist.all_gather_into_tensor(out, inp, group=group)
    elif out.is_cuda:  # gloo over device tensors (multi-process tests on one GPU): stage through the host
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather(list(host.chunk(dist.get_world_size(group))), inp.cpu(), group=group)
        out.copy_(host)
    else:  # gloo (CPU tests)
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), inp, group=group)


def gather_rows(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather row shards (produced with ``shard_bounds``) into the full [total, ...] tensor."""
    world = dist.get_world_size(group)
    counts = [shard_bounds(total, world, r)[1] - shard_bounds(total, world, r)[0] for r in range(world)]
    rank = dist.get_rank(group)
    if local.size(0) != counts[rank]:
        raise ValueError(f"rank {rank} holds {local.size(0)} rows, expected {counts[rank]}")
    width = max(counts) if counts else 0
    if all(c == width for c in counts):
        out = torch.empty((total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        _all_gather(out, local.contiguous(), group)
        return out
    pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.size(0)] = local
    buf = torch.empty((world * width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    _all_gather(buf, pad, group)
    return torch.cat([buf[r * width: r * width + counts[r]] for r in range(world)], dim=0)


def pack_rows(*tensors: torch.Tensor) -> Tuple[torch.Tensor, list]:
    """Row-wise byte packing of several [n, ...] tensors into one [n, W] int32 tensor (each row: the
    rows of ``tensors`` in order, reinterpreted as 32-bit words), so that ONE all-gather moves them
    all.  Returns the packed tensor and the spec ``unpack_rows`` needs.  Every element size must be a
    multiple of 4 bytes (int64 ids, fp32 alpha / beta)."""
    if not tensors:
        raise ValueError("pack_rows needs at least one tensor")
    n = tensors[0].size(0)
    cols, spec = [], []
    for t in tensors:
        if t.size(0) != n:
            raise ValueError("pack_rows: every tensor needs the same number of rows")
        if t.element_size() % 4:
            raise ValueError(f"pack_rows: {t.dtype} is not a multiple of 32 bits")
        # explicit row width: view(0, -1) is ambiguous for torch, and a rank may hold 0 rows when the
        # batch is smaller than the world (the other ranks would then wait in the all-gather forever)
        width = math.prod(t.shape[1:]) * t.element_size() // 4
        words = t.contiguous().reshape(n, -1 if n else 0).view(torch.int32).reshape(n, width)
        cols.append(words)
        spec.append((t.dtype, tuple(t.shape[1:]), words.size(1)))
    return torch.cat(cols, dim=1).contiguous(), spec


def unpack_rows(packed: torch.Tensor, spec: list) -> List[torch.Tensor]:
    """Inverse of ``pack_rows`` over any number of rows (e.g. the gathered [total, W] buffer):
    bit-exact views of the original dtypes and shapes."""
    out, c = [], 0
    n = packed.size(0)
    for dtype, shape, w in spec:
        words = packed[:, c:c + w].contiguous()
        out.append(words.view(dtype).view((n,) + shape))
        c += w
    return out


def local_rows(images: torch.Tensor, group=None) -> torch.Tensor:
    """This rank's contiguous row block of a batch every rank holds in full."""
    lo, hi = shard_bounds(images.size(0), dist.get_world_size(group), dist.get_rank(group))
    return images[lo:hi]


def sharded_sampler(decode: Callable[[torch.Tensor, int], Tuple[torch.Tensor, ...]], images_local: torch.Tensor,
                    total: int, max_len: int, group=None, gather_attention: bool = False):
    """Decode this rank's rows with ``decode(images, max_len) -> (ids, alpha, beta)`` and all-gather
    the ids (and optionally alpha/beta) to every rank.  ``images_local`` is the rank's
    ``shard_bounds(total, world, rank)`` block of the ``total``-row batch.  With ``gather_attention``
    the three outputs travel packed row by row in one int32 buffer (``pack_rows``): still ONE
    all-gather per call."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_bounds(total, world, rank)
    if images_local.size(0) != hi - lo:
        raise ValueError(f"rank {rank} was given {images_local.size(0)} rows, its shard of {total} is {hi - lo}")
    ids, alpha, beta = decode(images_local, max_len)
    if not gather_attention:
        return gather_rows(ids, total, group), None, None
    packed, spec = pack_rows(ids, alpha, beta)
    ids_all, alpha_all, beta_all = unpack_rows(gather_rows(packed, total, group), spec)
    return ids_all, alpha_all, beta_all

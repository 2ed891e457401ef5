"""CPU, world_size 2 (gloo): the sharded decode + one all-gather of ids reproduces the full-batch
decode exactly, for even and uneven shards.  The per-rank decoder here is the CPU oracle (this
exercises the sharding/gather logic of adaptive_amd.distributed; the GPU path runs the same code
over RCCL in bench.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from adaptive_amd import synth
from adaptive_amd import distributed as D
from adaptive_amd.distributed import gather_rows, pack_rows, shard_bounds, sharded_sampler, unpack_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_bounds():
    assert [shard_bounds(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    assert [shard_bounds(4096, 8, r) for r in range(8)][-1] == (3584, 4096)
    assert shard_bounds(1, 2, 1) == (1, 1)
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def test_pack_rows_layout_and_round_trip():
    """The packed all-gather buffer: row r holds row r's int64 ids (two int32 words each), then its
    alpha, then its beta, as raw 32-bit words; unpacking any row range gives the tensors back bit for
    bit (NaN payloads and -0.0 included)."""
    n, T = 3, 4
    ids = torch.arange(n * T, dtype=torch.int64).view(n, T) * (1 << 33) + 7
    alpha = torch.randn(n, T, 49)
    alpha[1, 2, 3] = float("nan")
    alpha[2, 0, 0] = -0.0
    beta = torch.rand(n, T, 1)
    packed, spec = pack_rows(ids, alpha, beta)
    assert packed.dtype == torch.int32 and packed.shape == (n, 2 * T + 49 * T + T)
    for r in range(n):
        assert torch.equal(packed[r, :2 * T], ids[r].view(torch.int32))
        assert torch.equal(packed[r, 2 * T:2 * T + 49 * T], alpha[r].reshape(-1).view(torch.int32))
        assert torch.equal(packed[r, 2 * T + 49 * T:], beta[r].reshape(-1).view(torch.int32))
    both = torch.cat([packed, packed[:2]])  # e.g. a gathered buffer of 5 rows
    i2, a2, b2 = unpack_rows(both, spec)
    assert i2.shape == (5, T) and a2.shape == (5, T, 49) and b2.shape == (5, T, 1)
    assert torch.equal(i2[:n], ids) and torch.equal(b2[:n], beta)
    assert torch.equal(a2[:n].view(torch.int32), alpha.view(torch.int32))
    with pytest.raises(ValueError):
        pack_rows(torch.zeros(2, 3, dtype=torch.int16))


def _worker(rank, world, port, total, T, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        from oracle.adaptive_oracle import OracleModel
        m = OracleModel(synth.make_weights(123))
        lo, hi = shard_bounds(total, world, rank)
        feats = torch.from_numpy(synth.make_features(hi - lo, seed=0, row0=lo))  # each rank makes only its rows
        calls = []
        real = D._all_gather
        D._all_gather = lambda out, inp, group: (calls.append(tuple(inp.shape)), real(out, inp, group))
        def decode(x, t):  # an empty shard (total < world) decodes to empty outputs, as the HIP path does
            if x.size(0) == 0:
                return (torch.empty(0, t, dtype=torch.int64), torch.empty(0, t, 49), torch.empty(0, t, 1))
            return m.sampler(x, max_len=t)
        try:
            ids, alpha, beta = sharded_sampler(decode, feats, total, T, gather_attention=True)
        finally:
            D._all_gather = real
        assert len(calls) == 1, calls  # ids, alpha and beta in ONE collective
        x = gather_rows(torch.arange(lo, hi, dtype=torch.int64).view(-1, 1), total)
        if rank == 0:  # by value (numpy): a tensor would travel as a shared-memory fd that this process
            q.put(tuple(v.numpy() for v in (ids, alpha, beta, x)))  # may close before the parent opens it
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 5, 1])
def test_sharded_decode_equals_full_batch(total):
    """total = 1 < world: rank 1 holds no rows and still joins the one all-gather."""
    world, T = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, PORTS[total], total, T, q))
             for r in range(world)]
    for p in procs:
        p.start()
    ids, alpha, beta, x = (torch.from_numpy(v) for v in q.get(timeout=300))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from oracle.adaptive_oracle import OracleModel
    r_ids, r_alpha, r_beta = OracleModel(synth.make_weights(123)).sampler(
        torch.from_numpy(synth.make_features(total)), max_len=T)
    assert torch.equal(x.view(-1), torch.arange(total))
    assert torch.equal(ids, r_ids)
    # the CPU oracle itself is not bitwise batch/thread-invariant (MKL blocking): compare closely
    torch.testing.assert_close(alpha, r_alpha, atol=1e-6, rtol=0)
    torch.testing.assert_close(beta, r_beta, atol=1e-6, rtol=0)


PORTS = {6: _free_port(), 5: _free_port(), 1: _free_port()}

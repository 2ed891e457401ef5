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
from adaptive_amd.distributed import gather_rows, shard_bounds, sharded_sampler


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
        ids, alpha, beta = sharded_sampler(lambda x, t: m.sampler(x, max_len=t), feats, total, T,
                                           gather_attention=True)
        x = gather_rows(torch.arange(lo, hi, dtype=torch.int64).view(-1, 1), total)
        if rank == 0:
            q.put((ids, alpha, beta, x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 5])
def test_sharded_decode_equals_full_batch(total):
    world, T = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, PORTS[total], total, T, q))
             for r in range(world)]
    for p in procs:
        p.start()
    ids, alpha, beta, x = q.get(timeout=300)
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


PORTS = {6: _free_port(), 5: _free_port()}

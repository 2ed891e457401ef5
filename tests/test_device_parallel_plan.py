"""CPU: the shard/gather plan of the single-process multi-device sampler (adaptive_amd/device_parallel.py)
and the device selection that mirrors the reference's ``torch.cuda.device_count() > 1`` test
(code_src/models/adaptive_attention.py:178-181)."""
import pytest
import torch

from adaptive_amd.device_parallel import plan_shards
from adaptive_amd.distributed import shard_bounds


@pytest.mark.parametrize("B,n", [(512, 8), (4096, 8), (513, 8), (7, 8), (1, 3), (0, 2), (100, 1), (301, 3)])
def test_blocks_cover_rows_once_in_order(B, n):
    devs = list(range(n))
    shards = plan_shards(B, devs)
    rows = [r for _, lo, hi in shards for r in range(lo, hi)]
    assert rows == list(range(B))                      # contiguous, in order, every row once
    assert all(hi > lo for _, lo, hi in shards)        # no empty block is launched
    sizes = [hi - lo for _, lo, hi in shards]
    assert not sizes or max(sizes) - min(sizes) <= 1   # balanced
    # same blocks as the one-process-per-GPU path (distributed.shard_bounds), device i <-> rank i
    for d, lo, hi in shards:
        assert (lo, hi) == shard_bounds(B, n, d)
    if B >= n:
        assert [d for d, _, _ in shards] == devs and shards[0][0] == devs[0]


def test_repeated_device_is_allowed():
    assert plan_shards(10, [0, 0, 0]) == [(0, 0, 4), (0, 4, 7), (0, 7, 10)]


def test_errors():
    with pytest.raises(ValueError):
        plan_shards(4, [])
    with pytest.raises(ValueError):
        plan_shards(-1, [0])


class _FakeImages:
    is_cuda = True

    def __init__(self, index):
        self.device = torch.device("cuda", index)


@pytest.mark.parametrize("mode,count,multi_rank,want", [
    (None, 1, False, None),                 # opt-in: off by default
    (None, 8, False, None),
    (False, 8, False, None),
    (True, 8, False, [2, 0, 1, 3, 4, 5, 6, 7]),  # every visible device, the images' own first
    (True, 3, False, [2, 0, 1]),
    (True, 2, True, [2, 0, 1]),             # explicit: all visible devices even under a process group
    ([2, 5], 8, False, [2, 5]),
    ([2], 8, False, None),
])
def test_device_selection(monkeypatch, mode, count, multi_rank, want):
    from adaptive_amd import Config, Encoder2Decoder
    monkeypatch.setattr(torch.cuda, "device_count", lambda: count)
    m = Encoder2Decoder(Config(adaptive_word_embed_size=32, adaptive_lstm_hidden_size=256, vocab_length=10))
    m.device_parallel = mode
    assert m._parallel_devices(_FakeImages(2), multi_rank) == want

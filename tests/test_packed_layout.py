"""CPU: the packed batch sizes Encoder2Decoder.forward caches per lengths list
(adaptive_attention.packed_batch_sizes) equal torch's pack_padded_sequence batch_sizes, and bad
lengths raise as the reference's packing does."""
import numpy as np
import pytest
import torch
from torch.nn.utils.rnn import pack_padded_sequence

from adaptive_amd.adaptive_attention import packed_batch_sizes


@pytest.mark.parametrize("seed", range(6))
def test_packed_batch_sizes_match_torch(seed):
    rng = np.random.default_rng(seed)
    B = int(rng.integers(1, 140))
    T = int(rng.integers(1, 25))
    lengths = sorted(rng.integers(1, T + 1, size=B).tolist(), reverse=True)
    ref = pack_padded_sequence(torch.zeros(B, max(lengths)), lengths, batch_first=True).batch_sizes
    assert packed_batch_sizes(lengths) == ref.tolist()
    assert sum(packed_batch_sizes(lengths)) == sum(lengths)


@pytest.mark.parametrize("bad", [[3, 0], [2, 3], [], [-1]])
def test_packed_batch_sizes_rejects_bad_lengths(bad):
    with pytest.raises(ValueError):
        packed_batch_sizes(bad)

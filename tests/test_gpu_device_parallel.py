"""GPU: the single-process multi-device sampler (adaptive_amd/device_parallel.py), the counterpart of
the reference's ``torch.cuda.device_count() > 1`` -> nn.DataParallel sampler
(code_src/models/adaptive_attention.py:178-181).

A one-GPU box cannot place blocks on other GPUs, so the multi-device code path runs here with the
same device listed more than once: every block but the first goes through the remote-device
machinery (its own role stream, a DecodePlan over buffers it owns, stream-local peer copies in and
out, event hand-back to the caller's stream).  On one visible device the default (``None``, as the
reference) reduces to today's single-device decode.  N > 1 real devices are unmeasured here.
"""
import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder, synth
from adaptive_amd.adaptive_attention import synthetic_features

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(gpu_device):
    return Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)


def test_default_reduces_to_single_device(model, gpu_device):
    if torch.cuda.device_count() != 1:
        pytest.skip("needs exactly one visible device")
    assert model._parallel_devices(synthetic_features(4, gpu_device, seed=0), False) is None
    feats = synthetic_features(96, gpu_device, seed=1)
    a = model.sampler(feats, max_len=10)
    model.device_parallel = False
    try:
        b = model.sampler(feats, max_len=10)
    finally:
        model.device_parallel = None
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("devices,B,exact", [([0, 0], 512, False), ([0, 0, 0], 301, False), ([0, 0, 0, 0], 70, True),
                                             ([0, 0], 1, False)])
def test_blocks_through_remote_path_equal_one_decode(model, gpu_device, devices, B, exact):
    feats = synthetic_features(B, gpu_device, seed=7)
    ref = model.sampler(feats, max_len=14, exact_vocab=exact)
    model.device_parallel = devices
    try:
        for _ in range(2):  # first call captures the blocks' plans, second replays them
            got = model.sampler(feats, max_len=14, exact_vocab=exact)
            for x, y in zip(ref, got):
                assert torch.equal(x, y)
    finally:
        model.device_parallel = None


def test_remote_path_follows_weight_changes(gpu_device):
    """A replica re-packs (and drops its plans) when the model's parameters change."""
    m = Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)
    m.device_parallel = [0, 0]
    feats = torch.from_numpy(synth.make_features(40, seed=2)).to(gpu_device)
    a = m.sampler(feats, max_len=6)
    m.load_synthetic(99, bias_noise=0.02)
    b = m.sampler(feats, max_len=6)
    m.device_parallel = False
    ref = m.sampler(feats, max_len=6)
    for x, y in zip(ref, b):
        assert torch.equal(x, y)
    assert not torch.equal(a[0], b[0])

"""GPU: the single-process multi-device sampler (adaptive_amd/device_parallel.py), the counterpart of
the reference's ``torch.cuda.device_count() > 1`` -> nn.DataParallel sampler
(code_src/models/adaptive_attention.py:178-181).

A one-GPU box cannot place blocks on other GPUs, so the multi-device code path runs here with the
same device listed more than once and ``device_parallel.FORCE_REMOTE`` set: every block but the
first then goes through the remote-device machinery -- a weight replica packed by
``aa_pack_weights`` into its own buffer, a ``_ReplicaView`` DecodePlan over the replica's weights,
its own role stream, stream-local copies in and out (hipMemcpyAsync), event hand-back to the
caller's stream.  Without FORCE_REMOTE the repeated device is the home device and its extra blocks
run ``DecodePlan(owner)`` instead (also tested).  The mode is opt-in; N > 1 real devices are
unmeasured here.
"""
import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder, device_parallel, synth
from adaptive_amd.adaptive_attention import synthetic_features

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(gpu_device):
    return Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)


def test_default_is_single_device(model, gpu_device):
    assert model.device_parallel is False  # opt-in
    assert model._parallel_devices(synthetic_features(4, gpu_device, seed=0), False) is None
    if torch.cuda.device_count() != 1:
        return
    feats = synthetic_features(96, gpu_device, seed=1)
    a = model.sampler(feats, max_len=10)
    model.device_parallel = True  # one visible device: reduces to the plain decode
    try:
        b = model.sampler(feats, max_len=10)
    finally:
        model.device_parallel = False
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.fixture(params=[True, False], ids=["force_remote", "home_plans"])
def force_remote(request):
    device_parallel.FORCE_REMOTE = request.param
    yield request.param
    device_parallel.FORCE_REMOTE = False


@pytest.mark.parametrize("devices,B,exact", [([0, 0], 512, False), ([0, 0, 0], 301, False), ([0, 0, 0, 0], 70, True),
                                             ([0, 0], 1, False)])
def test_blocks_through_remote_path_equal_one_decode(gpu_device, devices, B, exact, force_remote):
    m = Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)
    feats = synthetic_features(B, gpu_device, seed=7)
    ref = m.sampler(feats, max_len=14, exact_vocab=exact)
    m.device_parallel = devices
    for _ in range(2):  # first call captures the blocks' plans, second replays them
        got = m.sampler(feats, max_len=14, exact_vocab=exact)
        for x, y in zip(ref, got):
            assert torch.equal(x, y)
    reps = [r for d, r in m._replicas.items()]
    if len(devices) > 1 and B > 1:
        assert reps and all(r.home is (not force_remote) for r in reps)
        if force_remote:  # the replica packed its own copy of the weights
            assert all(r.packed is not None and r.packed.data_ptr() != m._packed.data_ptr() for r in reps)


def test_remote_path_follows_weight_changes(gpu_device):
    """A replica re-packs (and drops its plans) when the model's parameters change."""
    m = Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)
    m.device_parallel = [0, 0]
    device_parallel.FORCE_REMOTE = True
    try:
        feats = torch.from_numpy(synth.make_features(40, seed=2)).to(gpu_device)
        a = m.sampler(feats, max_len=6)
        m.load_synthetic(99, bias_noise=0.02)
        b = m.sampler(feats, max_len=6)
    finally:
        device_parallel.FORCE_REMOTE = False
    m.device_parallel = False
    ref = m.sampler(feats, max_len=6)
    for x, y in zip(ref, b):
        assert torch.equal(x, y)
    assert not torch.equal(a[0], b[0])

"""GPU: the ResNet-152 trunk path — images [B,3,224,224] -> MIOpen trunk ->
HIP decode, and training through the trunk (the HIP backward hands dL/dA to the trunk's autograd).
The trunk is PyTorch-ROCm library code: it is checked against the same module on the CPU with a
relative tolerance (convolution algorithms differ); the decode after it is the tested HIP path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence

from adaptive_amd import Config, Encoder2Decoder

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return (torch.linalg.norm(a.double() - b.double()) / torch.linalg.norm(b.double())).item()


@pytest.fixture(scope="module")
def tmodel(gpu_device):
    torch.manual_seed(0)
    m = Encoder2Decoder(Config(), trunk=True).load_synthetic(123)
    with torch.no_grad():  # scale the trunk so activations stay O(1) through 50 blocks
        for mod in m.encoder.resnet_conv.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.2, 0.4)
                mod.running_var.uniform_(0.8, 1.2)
    return m.to(gpu_device).eval()


def test_trunk_features_match_cpu(tmodel, gpu_device):
    x = torch.rand(2, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    cpu_trunk = Encoder2Decoder(Config(), trunk=True)
    cpu_trunk.load_state_dict({k: v.cpu() for k, v in tmodel.state_dict().items()})
    cpu_trunk.eval()
    with torch.no_grad():
        ref = cpu_trunk.encoder.resnet_conv(x)
    got = tmodel.features(x.to(gpu_device)).cpu()
    assert got.shape == (2, 2048, 7, 7)
    assert _rel(got, ref) < 1e-4
    tmodel.trunk_fold = False
    unfolded = tmodel.features(x.to(gpu_device)).cpu()
    tmodel.trunk_fold = True
    assert _rel(unfolded, ref) < 1e-4


def test_sampler_on_images_equals_sampler_on_features(tmodel, gpu_device):
    """(MIOpen may pick a different convolution algorithm on a later call, so the features of two
    trunk runs agree to rounding, not bit for bit: ids equal, alpha / beta to 1e-5.)"""
    x = torch.rand(3, 3, 224, 224, generator=torch.Generator().manual_seed(2)).to(gpu_device)
    ids, alpha, beta = tmodel.sampler(x, max_len=12)
    with torch.no_grad():
        feats = tmodel.features(x)
    ids2, alpha2, beta2 = tmodel.sampler(feats, max_len=12)
    assert torch.equal(ids, ids2)
    torch.testing.assert_close(alpha, alpha2, atol=1e-5, rtol=0)
    torch.testing.assert_close(beta, beta2, atol=1e-5, rtol=0)
    b_ids = tmodel.beam_search(x, 12, 3)[0]
    assert b_ids.shape == (3, 12)


def _step(m, x, caps, lengths):
    m.zero_grad()
    packed = m(x, caps, lengths)
    tgt = pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0]
    loss = F.cross_entropy(packed[0], tgt)
    loss.backward()
    return loss


CAPS = torch.tensor([[1, 5, 9, 13, 17, 0], [1, 6, 10, 14, 0, 0]], dtype=torch.int64)
LENGTHS = [5, 4]


def test_training_through_trunk_eval_bn_vs_cpu(tmodel, gpu_device):
    """Gradients reach the trunk (train.py:89 fine-tunes resnet_conv children >= 5) and, with the
    BatchNorms frozen (eval mode: a well-conditioned linear chain), match the CPU autograd of the
    same trunk feeding the CPU oracle."""
    from oracle.adaptive_oracle import TrainOracle
    x = torch.rand(2, 3, 224, 224, generator=torch.Generator().manual_seed(3))
    m = tmodel.eval()
    loss = _step(m, x.to(gpu_device), CAPS.to(gpu_device), LENGTHS)
    cpu = Encoder2Decoder(Config(), trunk=True)
    cpu.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    trunk = cpu.encoder.resnet_conv.eval()
    sd = {k: v.detach().numpy() for k, v in cpu.state_dict().items() if not k.startswith("encoder.resnet_conv.")}
    rloss, _ = TrainOracle(sd).loss(trunk(x), CAPS, LENGTHS)
    rloss.backward()
    assert abs(loss.item() - rloss.item()) <= 1e-4 * abs(rloss.item())
    for name in ("7.2.conv3.weight", "6.20.conv2.weight", "5.0.conv1.weight", "0.weight"):
        got = m.encoder.resnet_conv.get_parameter(name).grad.cpu()
        assert _rel(got, trunk.get_parameter(name).grad) < 1e-3, name


def test_training_through_trunk_train_bn(tmodel, gpu_device):
    """Train-mode BatchNorm (batch statistics, as train.py runs it) through the whole pipeline:
    forward + backward complete and every fine-tuned child (>= 5, cfg
    opt_fine_tune_cnn_start_layer) receives a finite, non-zero gradient.  (Values are compared in
    the eval-BN test above: with batch statistics at B = 2 the trunk's gradient is so
    ill-conditioned that MIOpen's non-deterministic weight-gradient reductions alone move it by
    several % run to run.)"""
    x = torch.rand(2, 3, 224, 224, generator=torch.Generator().manual_seed(3)).to(gpu_device)
    m = tmodel
    state = {k: v.clone() for k, v in m.state_dict().items()}
    m.train()
    try:
        loss = _step(m, x, CAPS.to(gpu_device), LENGTHS)
        assert torch.isfinite(loss)
        for n, p in m.encoder.resnet_conv.named_parameters():
            if int(n.split(".")[0]) >= 5:
                assert torch.isfinite(p.grad).all() and p.grad.abs().max() > 0, n
    finally:
        m.load_state_dict(state)  # undo the running-statistics update
        m.eval()

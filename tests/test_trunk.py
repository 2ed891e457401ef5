"""CPU: the ResNet-152 trunk (adaptive_amd/trunk.py) has the reference's
module layout — list(torchvision resnet152().children())[:-2], baseline_attention.py:16-18 — so
reference checkpoints (trunk keys included) load strictly, and its BatchNorm-folded inference copy
computes the same function."""
import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder
from adaptive_amd.trunk import fold_bn, resnet_conv


@pytest.fixture(scope="module")
def trunk():
    torch.manual_seed(0)
    m = resnet_conv().eval()
    with torch.no_grad():  # non-trivial running statistics so folding is exercised
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
                mod.weight.uniform_(0.2, 0.6)
                mod.bias.uniform_(-0.1, 0.1)
    return m


def test_layout_matches_torchvision_resnet152(trunk):
    sd = trunk.state_dict()
    # torchvision resnet152: 60,192,808 parameters, minus fc (2048*1000 + 1000)
    assert sum(p.numel() for p in trunk.parameters()) == 60_192_808 - 2_049_000
    assert len(sd) == 932 - 2
    assert [len(trunk[i]) for i in range(4, 8)] == [3, 8, 36, 3]
    assert tuple(sd["0.weight"].shape) == (64, 3, 7, 7)
    assert tuple(sd["4.0.downsample.0.weight"].shape) == (256, 64, 1, 1)
    assert tuple(sd["5.0.conv2.weight"].shape) == (128, 128, 3, 3) and trunk[5][0].conv2.stride == (2, 2)
    assert tuple(sd["7.2.conv3.weight"].shape) == (2048, 512, 1, 1)
    assert "7.2.bn3.num_batches_tracked" in sd


def test_folded_trunk_equals_eval_trunk(trunk):
    x = torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        a = trunk(x)
        b = fold_bn(trunk)(x.contiguous(memory_format=torch.channels_last))
    assert a.shape == (1, 2048, 7, 7)
    assert torch.linalg.norm(a - b) <= 1e-5 * torch.linalg.norm(a)


def test_model_with_trunk_loads_reference_checkpoint(trunk, manifest):
    m = Encoder2Decoder(Config(), trunk=True)
    sd = m.state_dict()
    decode_keys = {k for k in sd if not k.startswith("encoder.resnet_conv.")}
    assert decode_keys == set(manifest["state_dict"])
    assert {k[len("encoder.resnet_conv."):] for k in sd if k.startswith("encoder.resnet_conv.")} == set(trunk.state_dict())
    ref = Encoder2Decoder(Config()).load_synthetic(3).state_dict()
    ref.update({"encoder.resnet_conv." + k: v for k, v in trunk.state_dict().items()})
    m.load_state_dict(ref)  # strict: a full reference checkpoint
    assert torch.equal(m.encoder.resnet_conv[7][2].conv3.weight, trunk[7][2].conv3.weight)
    with pytest.raises(RuntimeError):
        m.load_state_dict({k: v for k, v in ref.items() if not k.startswith("encoder.resnet_conv.7.")})

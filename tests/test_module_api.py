"""CPU: the drop-in module mirrors the reference surface (state-dict keys and shapes, attribute
tree, call signatures) and refuses to run anywhere but the HIP path."""
import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder


@pytest.fixture(scope="module")
def model():
    return Encoder2Decoder(Config())


def test_state_dict_matches_reference(model, manifest):
    ref = manifest["state_dict"]
    ours = {k: list(v.shape) for k, v in model.state_dict().items()}
    assert ours == ref


def test_attribute_tree(model):
    # what callers touch: model_factory.py:35,63-64; train.py:129,214
    assert list(model.encoder.resnet_conv.children()) == []
    assert len(list(model.encoder.affine_a.parameters())) == 2
    assert len(list(model.decoder.LSTM.parameters())) == 4
    assert model.decoder.adaptive.atten.affine_h.weight.shape == (1, 49)
    assert sum(p.numel() for p in model.decoder.parameters()) > 10_000_000


def test_reference_style_init(model):
    b = model.decoder.LSTM.bias_ih_l0.detach()
    assert torch.all(b[512:1024] == 0.5) and torch.all(b[:512] == 0)   # model_utils.py:69-71
    assert torch.all(model.decoder.adaptive.mlp.bias == 0)


def test_load_synthetic_and_checkpoint_with_trunk_keys():
    m = Encoder2Decoder(Config()).load_synthetic(123)
    sd = m.state_dict()
    sd["encoder.resnet_conv.0.weight"] = torch.zeros(1)  # a real checkpoint carries the trunk
    m2 = Encoder2Decoder(Config())
    m2.load_state_dict(sd)
    assert torch.equal(m2.decoder.adaptive.mlp.weight, m.decoder.adaptive.mlp.weight)


def test_cpu_tensors_are_rejected(model):
    with pytest.raises(RuntimeError, match="GPU|CUDA"):
        model.sampler(torch.zeros(2, 2048, 7, 7))


def test_teacher_forcing_has_no_cpu_path(model):
    with pytest.raises(RuntimeError, match="GPU|CUDA"):
        model(torch.zeros(2, 2048, 7, 7), torch.zeros(2, 5, dtype=torch.long), [4, 3])

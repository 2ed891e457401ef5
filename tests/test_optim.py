"""CPU: host logic of adaptive_amd.optim (the CrossEntropyLoss / Adam of train.py's closure,
train.py:63,197-219, model_factory.py:71) and the argument checks of their C-ABI entry points --
no device work (there is no GPU here).  The numerics are tests/test_gpu_optim.py."""
import pytest
import torch


@pytest.fixture(scope="module")
def lib():
    from adaptive_amd import _lib
    return _lib.load()


def test_adam_constructor_validation():
    from adaptive_amd.optim import Adam
    p = [torch.nn.Parameter(torch.zeros(3))]
    with pytest.raises(NotImplementedError):
        Adam(p, amsgrad=True)
    with pytest.raises(ValueError):
        Adam(p, lr=-1.0)
    with pytest.raises(ValueError):
        Adam(p, betas=(1.0, 0.999))
    opt = Adam(p, lr=1e-4, betas=(0.8, 0.999), weight_decay=1e-4)
    g = opt.param_groups[0]
    assert (g["lr"], g["betas"], g["weight_decay"], g["amsgrad"]) == (1e-4, (0.8, 0.999), 1e-4, False)
    # same hyper-parameter keys as torch's Adam, so state dicts move between the two
    assert set(torch.optim.Adam(p).param_groups[0]) <= set(g) | {"decoupled_weight_decay"}


def test_adam_fails_loudly_on_cpu_tensors(lib):
    from adaptive_amd.optim import Adam
    p = torch.nn.Parameter(torch.zeros(8))
    p.grad = torch.ones(8)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        Adam([p]).step()
    Adam([torch.nn.Parameter(torch.zeros(8))]).step()  # no gradients: nothing to do, no error


def test_cross_entropy_fails_loudly_on_cpu_tensors(lib):
    from adaptive_amd.optim import CrossEntropyLoss, cross_entropy
    with pytest.raises(RuntimeError, match="GPU tensor"):
        cross_entropy(torch.zeros(4, 10), torch.zeros(4, dtype=torch.int64))
    with pytest.raises(NotImplementedError):
        CrossEntropyLoss(reduction="sum")


def test_capi_argument_errors(lib):
    from adaptive_amd import _lib
    t = (_lib.AdamTensor * 1)(_lib.AdamTensor(256, 512, 768, 1024, 10))
    assert lib.aa_adam_step(None, -1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -3
    assert lib.aa_adam_step(None, 1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1
    assert lib.aa_adam_step(t, 1, 0.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -3      # step counts from 1
    assert lib.aa_adam_step(None, 0, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == 0      # nothing to do
    bad = (_lib.AdamTensor * 1)(_lib.AdamTensor(256, None, 768, 1024, 10))
    assert lib.aa_adam_step(bad, 1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1
    neg = (_lib.AdamTensor * 1)(_lib.AdamTensor(256, 512, 768, 1024, -1))
    assert lib.aa_adam_step(neg, 1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -3
    empty = (_lib.AdamTensor * 1)(_lib.AdamTensor(None, None, None, None, 0))
    assert lib.aa_adam_step(empty, 1, 1.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == 0     # numel 0 skipped
    assert lib.aa_cross_entropy_workspace_bytes(10) == 120
    assert lib.aa_cross_entropy_workspace_bytes(0) == 0
    assert lib.aa_cross_entropy_forward(256, 0, 10, 10, 256, -100, 256, 256, 256, 0, None) == -3
    assert lib.aa_cross_entropy_forward(256, 4, 10, 9, 256, -100, 256, 256, 256, 48, None) == -3  # ldx < V
    assert lib.aa_cross_entropy_forward(256, 4, 10, 10, None, -100, 256, 256, 256, 48, None) == -1
    assert lib.aa_cross_entropy_forward(256, 4, 10, 10, 256, -100, 256, 256, 256, 47, None) == -4
    assert lib.aa_cross_entropy_backward(256, 4, 10, 10, 256, -100, 256, 256, 256, 48, None, 10, None) == -1
    assert lib.aa_cross_entropy_backward(256, 4, 10, 10, 256, -100, 256, 256, 256, 48, 512, 8, None) == -3
    # a workspace from a forward over fewer rows is refused
    assert lib.aa_cross_entropy_backward(256, 4, 10, 10, 256, -100, 256, 256, 256, 47, 512, 10, None) == -4
    # in place (dlogits == logits) only with the same pitch
    assert lib.aa_cross_entropy_backward(256, 4, 10, 10, 256, -100, 256, 256, 256, 48, 256, 12, None) == -3

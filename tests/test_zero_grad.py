"""Encoder2Decoder.zero_grad / adaptive_amd.optim.Adam.zero_grad fast paths (host logic, CPU): the
same parameters as torch's own, including ones registered after construction and shared modules."""
import torch

from adaptive_amd import Config, Encoder2Decoder
from adaptive_amd.optim import Adam


def _fill(params):
    for p in params:
        p.grad = torch.ones_like(p)


def test_model_zero_grad_covers_every_parameter():
    m = Encoder2Decoder(Config())
    m.extra = torch.nn.Linear(3, 2)                          # a module added after construction
    m.decoder.extra_p = torch.nn.Parameter(torch.zeros(4))   # a parameter on a submodule
    m.shared = m.decoder.LSTM                                # the same module reachable twice
    ps = list(m.parameters())
    _fill(ps)
    m.zero_grad()
    assert all(p.grad is None for p in ps)
    _fill(ps)
    m.zero_grad(set_to_none=False)                           # torch's own path
    assert all(p.grad is not None and not p.grad.any() for p in ps)


def test_adam_zero_grad_sets_none():
    ps = [torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2, 2))]
    opt = Adam(ps, lr=1e-3)
    _fill(ps)
    opt.zero_grad()
    assert all(p.grad is None for p in ps)
    _fill(ps)
    opt.zero_grad(set_to_none=False)
    assert all(p.grad is not None and not p.grad.any() for p in ps)

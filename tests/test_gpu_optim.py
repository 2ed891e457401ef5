"""GPU: adaptive_amd.optim against PyTorch's own ops on the same inputs -- the HIP cross entropy
(aa_cross_entropy_*) against F.cross_entropy (train.py:63,208), the HIP Adam (aa_adam_step)
against torch.optim.Adam (model_factory.py:71), and train.py's closure (train.py:197-219) with both
against the closure with torch's.  Tolerances: fp32, written per assertion (the two sides round
exp/log and the reductions in different orders; Adam is in torch's op order)."""
import copy
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _scores(dev, N, V, seed=0, scale=4.0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(N, V, generator=g) * scale).to(dev)
    t = torch.randint(0, V, (N,), generator=g).to(dev)
    return x, t


@pytest.mark.parametrize("N,V,ignore", [(1741, 10123, False), (1741, 10123, True), (5, 3, False), (300, 1, False),
                                        (64, 40000, True)])
def test_cross_entropy_matches_torch(gpu_device, N, V, ignore):
    from adaptive_amd.optim import cross_entropy
    x, t = _scores(gpu_device, N, V)
    if ignore:
        t[::7] = -100
    xa = x.clone().requires_grad_()
    xr = x.clone().requires_grad_()
    la = cross_entropy(xa, t)
    lr = F.cross_entropy(xr, t)
    (la * 1.7).backward()
    (lr * 1.7).backward()
    # fp32 sums of N row losses / V exponentials in different orders
    assert abs(la.item() - lr.item()) <= 1e-5 * abs(lr.item()) + 1e-7, (la.item(), lr.item())
    err = (xa.grad - xr.grad).abs().max().item()
    assert err <= 1e-5 * xr.grad.abs().max().item(), err
    assert torch.all(xa.grad[t == -100] == 0)


def test_cross_entropy_strided_input_deterministic_and_poisoned_target(gpu_device):
    from adaptive_amd.optim import CrossEntropyLoss
    wide, t = _scores(gpu_device, 257, 10200, seed=3)
    x = wide[:, :10123]  # row pitch 10200 > V: read in place, no copy
    t = t % 10123
    crit = CrossEntropyLoss()
    l1, l2 = crit(x, t), crit(x, t)
    assert l1.item() == l2.item()  # fixed-order reductions
    assert abs(l1.item() - F.cross_entropy(x, t).item()) <= 1e-5 * abs(l1.item())
    bad = t.clone()
    bad[5] = 10123
    assert torch.isnan(crit(x, bad)).item()


def _adam_pair(dev, n_extra=0):
    torch.manual_seed(0)
    shapes = [(10123, 512), (10123,), (2048, 768), (2048,), (49, 512), (7,), (1000, 3)] + [(33,)] * n_extra
    base = [torch.randn(s, device=dev) for s in shapes]
    buf = torch.randn(4097, device=dev)
    # the last parameter sits 4 bytes into its buffer: the kernel's unaligned (scalar) path
    pa = [b.clone().requires_grad_() for b in base] + [buf[1:].detach().requires_grad_()]
    pr = [p.detach().clone().requires_grad_() for p in pa]
    return pa, pr


@pytest.mark.parametrize("wd,betas,n_extra", [(0.0, (0.9, 0.999), 0), (1e-4, (0.8, 0.999), 0), (0.0, (0.9, 0.99), 30)])
def test_adam_matches_torch(gpu_device, wd, betas, n_extra):
    """HIP Adam vs torch.optim.Adam over four steps, PER ELEMENT: every moment and parameter entry
    within a rounding-error bound built from that entry's own magnitudes.  Each step adds, per
    element, a few fp32 unit roundoffs (u = 2^-24) of the operands of that step's ops (torch's
    compiled lerp / addcmul / addcdiv may contract into fmas that round once where this kernel rounds
    twice), and the parameter bound carries the moments' error bounds through the update
    p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)."""
    from adaptive_amd.optim import Adam
    u = 2.0 ** -24
    lr, eps = 1e-3, 1e-8
    b1, b2 = betas
    pa, pr = _adam_pair(gpu_device, n_extra)
    assert pa[-1].data_ptr() % 16 != 0
    oa = Adam(pa, lr=lr, betas=betas, weight_decay=wd)
    orf = torch.optim.Adam(pr, lr=lr, betas=betas, weight_decay=wd)
    g = torch.Generator(device=gpu_device).manual_seed(1)
    Em = [torch.zeros_like(r) for r in pr]
    Ev = [torch.zeros_like(r) for r in pr]
    Ep = [torch.zeros_like(r) for r in pr]
    worst = {"exp_avg": 0.0, "exp_avg_sq": 0.0, "param": 0.0}
    for step in range(4):
        for i, (a, r) in enumerate(zip(pa, pr)):
            gr = torch.randn(a.shape, device=gpu_device, generator=g) * 10.0 ** -(i % 3)
            a.grad, r.grad = gr.clone(), gr.clone()
        if step == 2:
            pa[1].grad = pr[1].grad = None  # a parameter without a gradient is left alone
        prev = [(orf.state[r]["exp_avg"].clone(), orf.state[r]["exp_avg_sq"].clone()) if r in orf.state
                else (torch.zeros_like(r), torch.zeros_like(r)) for r in pr]
        p_before = [r.detach().clone() for r in pr]
        oa.step()
        orf.step()
        for i, (a, r) in enumerate(zip(pa, pr)):
            sa, sr = oa.state[a], orf.state[r]
            assert float(sa["step"]) == float(sr["step"])
            if r.grad is None:
                continue
            t = float(sr["step"])
            gg = r.grad.abs() + wd * p_before[i].abs()  # the gradient as the update sees it
            m, v = sr["exp_avg"], sr["exp_avg_sq"]
            m0, v0 = prev[i]
            Em[i] = b1 * Em[i] + 4 * u * (m.abs() + (1 - b1) * gg + m0.abs())
            Ev[i] = b2 * Ev[i] + 4 * u * (v + (1 - b2) * gg * gg + v0)
            ss, bc2 = lr / (1 - b1 ** t), (1 - b2 ** t) ** 0.5
            sq = v.sqrt()
            d = sq / bc2 + eps
            dv = torch.where(sq > 0, Ev[i] / (2 * sq.clamp_min(1e-30) * bc2), Ev[i].sqrt() / bc2)
            Ep[i] = Ep[i] + 4 * u * r.detach().abs() + ss * (Em[i] / d + m.abs() * dv / (d * d) + 8 * u * m.abs() / d)
            for key, E in (("exp_avg", Em[i]), ("exp_avg_sq", Ev[i])):
                err = (sa[key] - sr[key]).abs()
                ratio = (err / E.clamp_min(1e-45)).max().item()
                worst[key] = max(worst[key], ratio)
                assert bool((err <= E).all()), (key, i, step, ratio)
            err = (a.detach() - r.detach()).abs()
            ratio = (err / Ep[i].clamp_min(1e-45)).max().item()
            worst["param"] = max(worst["param"], ratio)
            assert bool((err <= Ep[i]).all()), ("param", i, step, ratio)
    print("worst error / per-element bound:", worst)
    # the state dict moves to torch's Adam and back
    orf2 = torch.optim.Adam(pr, lr=1e-3, betas=betas, weight_decay=wd)
    orf2.load_state_dict(oa.state_dict())
    oa2 = Adam(pa, lr=1e-3, betas=betas, weight_decay=wd)
    oa2.load_state_dict(orf.state_dict())
    assert float(oa2.state[pa[0]]["step"]) == 4.0


def test_adam_reused_plan_and_state_reload(gpu_device):
    """The cached launch table (gradient tensors kept and overwritten in place, as
    zero_grad(set_to_none=False) leaves them) gives torch.optim.Adam's steps; load_state_dict then
    replaces the state tensors mid-run and the next steps use the loaded moments and counts."""
    from adaptive_amd.optim import Adam
    pa, pr = _adam_pair(gpu_device, 0)
    oa = Adam(pa, lr=1e-3)
    orf = torch.optim.Adam(pr, lr=1e-3)
    g = torch.Generator(device=gpu_device).manual_seed(2)
    for a, r in zip(pa, pr):
        a.grad, r.grad = torch.zeros_like(a), torch.zeros_like(r)
    for step in range(6):
        if step == 3:  # both reload the same state: torch's, after three steps
            sd = orf.state_dict()
            oa.load_state_dict(copy.deepcopy(sd))  # load_state_dict keeps CPU step tensors: no sharing
            orf.load_state_dict(copy.deepcopy(sd))
            for a, r in zip(pa, pr):
                a.data.copy_(r.data)
        for a, r in zip(pa, pr):
            gr = torch.randn(a.shape, device=gpu_device, generator=g)
            a.grad.copy_(gr)
            r.grad.copy_(gr)
        oa.step()
        orf.step()
        for a, r in zip(pa, pr):
            assert float(oa.state[a]["step"]) == float(orf.state[r]["step"]) == step + 1
            torch.testing.assert_close(a.detach(), r.detach(), rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(oa.state[a]["exp_avg_sq"], orf.state[r]["exp_avg_sq"], rtol=1e-5, atol=1e-12)


def test_train_closure_with_hip_loss_and_adam(gpu_device):
    """train.py:197-219 closure, three steps at B=16, T=10 (fp32 GEMMs, so that ulp-level
    differences are not amplified by bf16 operand rounding): HIP CrossEntropyLoss + clip_grad_norm_ + Adam against
    torch's on a second copy of the same model: the losses and parameters agree to fp32 rounding (the
    forward/backward kernels are the same, so only the loss and the update differ)."""
    from torch.nn.utils.rnn import pack_padded_sequence
    from adaptive_amd import Config, Encoder2Decoder
    from adaptive_amd.adaptive_attention import synthetic_features
    from adaptive_amd.optim import Adam, CrossEntropyLoss, clip_grad_norm_
    B, T = 16, 10
    rng = np.random.default_rng(0)
    lengths = sorted(rng.integers(T // 2, T + 1, size=B).tolist(), reverse=True)
    lengths[0] = T
    caps = torch.from_numpy(rng.integers(2, 10123, size=(B, T + 1))).to(gpu_device)
    caps[:, 0] = 1
    feats = synthetic_features(B, gpu_device, seed=0)
    targets = pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0]
    runs = []
    for hip in (True, False):
        model = Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)
        model.train_bf16 = False
        opt = (Adam if hip else torch.optim.Adam)(model.parameters(), lr=1e-3)
        crit = CrossEntropyLoss() if hip else torch.nn.CrossEntropyLoss()
        clip = clip_grad_norm_ if hip else torch.nn.utils.clip_grad_norm_
        losses = []
        for _ in range(3):
            model.zero_grad()
            opt.zero_grad()
            loss = crit(model(feats, caps, lengths)[0], targets)
            loss.backward()
            clip(model.decoder.LSTM.parameters(), 5.0)
            opt.step()
            losses.append(loss.item())
        runs.append((losses, {k: v.detach().clone() for k, v in model.state_dict().items()}))
    (la, sa), (lr, sr) = runs
    assert np.allclose(la, lr, rtol=1e-5, atol=0), (la, lr)
    for k in sr:
        err = (sa[k] - sr[k]).abs().max().item()
        assert err <= 2e-5 * max(1.0, sr[k].abs().max().item()), (k, err)


@pytest.mark.parametrize("max_norm", [5.0, 1e30, 0.0])
def test_clip_grad_norm_matches_torch(gpu_device, max_norm):
    """clip_grad_norm_ (train.py:213-214) vs torch.nn.utils.clip_grad_norm_: tensor sizes either side of
    the kernel's 8192-element chunk, an empty tensor, an unaligned view, a parameter without a
    gradient; the total norm to fp32 rounding (the sum order differs), the clipped gradients to a few
    ulps (the same multiply by a coefficient that differs by at most that), and no clip due leaves the
    gradients bit-identical (torch multiplies by exactly 1.0 then too).  New gradient tensors on the
    second call (the cached table takes their pointers)."""
    from adaptive_amd.optim import clip_grad_norm_
    buf = torch.empty(20001, device=gpu_device)
    shapes = [(4096, 1024), (4096,), (8192,), (8193,), (8191,), (1,), (0,), (3, 7)]
    for rep in range(2):
        torch.manual_seed(rep)
        pa = [torch.zeros(s, device=gpu_device, requires_grad=True) for s in shapes]
        pa.append(buf[1:].detach().requires_grad_())  # 4 bytes into its buffer: the scalar path
        pa.append(torch.zeros(5, device=gpu_device, requires_grad=True))  # no gradient
        for i, p in enumerate(pa[:-1]):
            p.grad = torch.randn(p.shape, device=gpu_device) * 10.0 ** -(i % 3)
        # the unaligned parameter's gradient is an unaligned view too (a fresh one on each call)
        pa[-2].grad = torch.empty(20001, device=gpu_device)[1:].copy_(pa[-2].grad)
        assert pa[-2].grad.data_ptr() % 16 != 0
        pr = [p.detach().clone().requires_grad_() for p in pa]
        for a, r in zip(pa, pr):
            r.grad = None if a.grad is None else a.grad.clone()
        ga0 = [None if p.grad is None else p.grad.clone() for p in pa]
        ta = clip_grad_norm_(pa, max_norm)
        tr = torch.nn.utils.clip_grad_norm_(pr, max_norm)
        assert ta.shape == () and ta.is_cuda and ta.dtype == torch.float32
        torch.testing.assert_close(ta, tr, rtol=1e-5, atol=0)
        for a, r, g0 in zip(pa, pr, ga0):
            if a.grad is None:
                assert r.grad is None
                continue
            if max_norm >= 1e30:
                assert torch.equal(a.grad, g0)
            else:
                torch.testing.assert_close(a.grad, r.grad, rtol=2e-5, atol=0)

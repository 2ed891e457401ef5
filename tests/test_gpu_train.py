"""Teacher-forced training step (Encoder2Decoder.forward + backward) on the GPU,
through the C-ABI (aa_train_forward / aa_train_backward), against the REAL reference's forward,
loss and gradients (tests/golden/train_b4.npz, made by tests/golden/make_golden_train.py) and
against the autograd of the CPU oracle on ragged batches.

Tolerances: the GPU path is fp32 with a different summation order than the reference's CPU
kernels, so packed scores agree to 1e-4 absolute, the loss to 1e-5 relative, and each gradient to
1e-3 relative (Frobenius) with every entry within 1e-2 of that parameter's largest gradient
magnitude.  (Entry-wise agreement is not tighter because a ReLU input within rounding of 0 can
take the other side of the kink: affine_a / affine_b gradients then differ in one row.)"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence

from conftest import load_golden

from adaptive_amd import Config, Encoder2Decoder, synth

pytestmark = pytest.mark.gpu

SCORE_TOL = 1e-4
GRAD_REL = 1e-3    # relative Frobenius error per parameter
GRAD_ENTRY = 1e-2  # max entry error / max |gradient|


def _grad_close(got, ref, name):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    assert np.abs(got - ref).max() <= GRAD_ENTRY * scale, name
    assert np.linalg.norm(got - ref) <= GRAD_REL * max(np.linalg.norm(ref), 1e-30), name


def _model(dev, seed=123, noise=0.02):
    return Encoder2Decoder(Config()).to(dev).load_synthetic(seed, bias_noise=noise)


def _loss(model, feats, caps, lengths):
    packed = model(feats, caps, lengths)
    targets = pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0]
    return F.cross_entropy(packed[0], targets), packed


def test_train_step_vs_reference_golden(gpu_device):
    g = load_golden("train_b4")
    model = _model(gpu_device)
    feats = torch.from_numpy(synth.make_features(4, seed=7)).to(gpu_device)
    caps = torch.from_numpy(g["captions"]).to(gpu_device)
    lengths = g["lengths"].tolist()
    loss, packed = _loss(model, feats, caps, lengths)
    assert packed[1].tolist() == g["batch_sizes"].tolist()
    np.testing.assert_allclose(packed[0].detach().cpu().numpy(), g["scores"], atol=SCORE_TOL, rtol=0)
    assert abs(loss.item() - float(g["loss"])) <= 1e-5 * abs(float(g["loss"]))
    model.zero_grad()
    loss.backward()
    for k, p in model.named_parameters():
        got = p.grad.detach().cpu().numpy().reshape(-1)
        ref = g["g:" + k]
        if "g:" + k + ":idx" in g:
            got_s = got[g["g:" + k + ":idx"]]
        else:
            got_s = got
        _grad_close(got_s, ref, k)
        ref_norm = float(g["g:" + k + ":norm"])
        assert abs(np.linalg.norm(got.astype(np.float64)) - ref_norm) <= 1e-4 * max(ref_norm, 1e-12), k


def test_train_step_vs_oracle_ragged(gpu_device):
    """B = 13, lengths with ties and a length-1 row, captions wider than T + 1."""
    from oracle.adaptive_oracle import TrainOracle
    B, L = 13, 12
    lengths = [9, 9, 8, 7, 7, 6, 5, 4, 4, 3, 2, 1, 1]
    rng = np.random.default_rng(5)
    caps_np = rng.integers(0, 10123, size=(B, L)).astype(np.int64)
    caps_np[:, 0] = 1
    state = synth.make_weights(31, bias_noise=0.01)
    feats_np = synth.make_features(B, seed=9)
    oracle = TrainOracle(state)
    rloss, rpacked = oracle.loss(torch.from_numpy(feats_np), torch.from_numpy(caps_np), lengths)
    rloss.backward()
    model = _model(gpu_device, seed=31, noise=0.01)
    loss, packed = _loss(model, torch.from_numpy(feats_np).to(gpu_device), torch.from_numpy(caps_np).to(gpu_device),
                         lengths)
    np.testing.assert_allclose(packed[0].detach().cpu().numpy(), rpacked[0].detach().numpy(), atol=SCORE_TOL, rtol=0)
    assert abs(loss.item() - rloss.item()) <= 1e-5 * abs(rloss.item())
    loss.backward()
    for k, p in model.named_parameters():
        got = p.grad.detach().cpu().numpy()
        _grad_close(got, oracle.w[k].grad.detach().numpy(), k)


def test_train_feature_gradient_vs_oracle(gpu_device):
    """dL/dA into the trunk's output (aa_train_backward's dfeats, CNN fine-tuning, train.py:89)
    against the oracle's autograd, on the ragged B = 13 batch."""
    from oracle.adaptive_oracle import TrainOracle
    B, L = 13, 12
    lengths = [9, 9, 8, 7, 7, 6, 5, 4, 4, 3, 2, 1, 1]
    rng = np.random.default_rng(5)
    caps_np = rng.integers(0, 10123, size=(B, L)).astype(np.int64)
    caps_np[:, 0] = 1
    state = synth.make_weights(31, bias_noise=0.01)
    feats_np = synth.make_features(B, seed=9)
    ref_feats = torch.from_numpy(feats_np).requires_grad_(True)
    rloss, _ = TrainOracle(state).loss(ref_feats, torch.from_numpy(caps_np), lengths)
    rloss.backward()
    model = _model(gpu_device, seed=31, noise=0.01)
    feats = torch.from_numpy(feats_np).to(gpu_device).requires_grad_(True)
    loss, _ = _loss(model, feats, torch.from_numpy(caps_np).to(gpu_device), lengths)
    loss.backward()
    # every V entry within rounding of the ReLU kink that lands on the other side moves a whole
    # W_a row (2048 entries) of dA, so the Frobenius bound is 3x the parameter-gradient one here
    got, ref = feats.grad.cpu().double().numpy(), ref_feats.grad.double().numpy()
    assert np.abs(got - ref).max() <= GRAD_ENTRY * np.abs(ref).max()
    assert np.linalg.norm(got - ref) <= 3 * GRAD_REL * np.linalg.norm(ref)


def test_train_step_deterministic(gpu_device):
    g = load_golden("train_b4")
    feats = torch.from_numpy(synth.make_features(4, seed=7)).to(gpu_device)
    caps = torch.from_numpy(g["captions"]).to(gpu_device)
    grads = []
    for _ in range(2):
        model = _model(gpu_device)
        loss, _ = _loss(model, feats, caps, g["lengths"].tolist())
        loss.backward()
        grads.append({k: p.grad.clone() for k, p in model.named_parameters()})
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


@pytest.mark.parametrize("bf16", [True, False])
def test_train_two_streams_bit_identical_to_one(gpu_device, bf16):
    """aa_train_forward_aux / aa_train_backward_aux (the V GEMM and the weight gradients on a second
    stream) against the one-stream calls: scores, every gradient and dL/dfeats bit for bit, on
    bench_train's B = 128, T = 18 batch (lengths T .. T/2)."""
    from bench_train import make_batch
    from adaptive_amd.adaptive_attention import synthetic_features
    caps_np, lengths = make_batch(128, 18)
    caps = torch.from_numpy(caps_np).to(gpu_device)
    out = []
    for two in (True, False):
        model = _model(gpu_device)
        model.train_bf16 = bf16
        model.train_aux_stream = two
        feats = synthetic_features(128, gpu_device, seed=3).requires_grad_(True)
        loss, packed = _loss(model, feats, caps, lengths)
        loss.backward()
        got = {k: p.grad.clone() for k, p in model.named_parameters()}
        got["scores"], got["dfeats"] = packed[0].detach().clone(), feats.grad.clone()
        out.append(got)
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_train_closure_adam_clip_reduces_loss(gpu_device):
    """train.py:197-219 as written: zero_grad, forward, CE, backward, clip LSTM grad norm, Adam step."""
    B, L = 8, 10
    lengths = [9, 8, 8, 6, 5, 5, 3, 2]
    rng = np.random.default_rng(11)
    caps = torch.from_numpy(rng.integers(0, 10123, size=(B, L)).astype(np.int64)).to(gpu_device)
    caps[:, 0] = 1
    feats = torch.from_numpy(synth.make_features(B, seed=3)).to(gpu_device)
    model = _model(gpu_device)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        model.zero_grad()
        opt.zero_grad()
        loss, _ = _loss(model, feats, caps, lengths)
        losses.append(loss.item())
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.decoder.LSTM.parameters(), 5.0)
        opt.step()
    assert losses[-1] < losses[0]


# bf16 GEMMs (AA_TRAIN_BF16, BASELINE config 5 "bf16 compute / fp32 master"): every GEMM operand is
# rounded to bf16 (unit roundoff 2^-8 = 3.9e-3) with fp32 accumulation, so a product carries a
# relative error of ~2 * 3.9e-3 / sqrt(averaging) per GEMM and the chain forward -> backward
# compounds a few of them.  Tolerances: packed scores within 2e-2 relative (Frobenius) of the fp32
# oracle, the loss within 1e-3 relative, each parameter gradient within 5e-2 relative (Frobenius).
BF16_SCORE_REL = 2e-2
BF16_LOSS_REL = 1e-3
BF16_GRAD_REL = 5e-2


def test_train_bf16_vs_oracle(gpu_device):
    from oracle.adaptive_oracle import TrainOracle
    B, L = 13, 12
    lengths = [9, 9, 8, 7, 7, 6, 5, 4, 4, 3, 2, 1, 1]
    rng = np.random.default_rng(5)
    caps_np = rng.integers(0, 10123, size=(B, L)).astype(np.int64)
    caps_np[:, 0] = 1
    state = synth.make_weights(31, bias_noise=0.01)
    feats_np = synth.make_features(B, seed=9)
    oracle = TrainOracle(state)
    rloss, rpacked = oracle.loss(torch.from_numpy(feats_np), torch.from_numpy(caps_np), lengths)
    rloss.backward()
    model = _model(gpu_device, seed=31, noise=0.01)
    model.train_bf16 = True
    loss, packed = _loss(model, torch.from_numpy(feats_np).to(gpu_device), torch.from_numpy(caps_np).to(gpu_device),
                         lengths)
    got = packed[0].detach().cpu().double().numpy()
    ref = rpacked[0].detach().double().numpy()
    assert np.linalg.norm(got - ref) <= BF16_SCORE_REL * np.linalg.norm(ref)
    assert abs(loss.item() - rloss.item()) <= BF16_LOSS_REL * abs(rloss.item())
    loss.backward()
    for k, p in model.named_parameters():
        g = p.grad.detach().cpu().double().numpy()
        r = oracle.w[k].grad.detach().double().numpy()
        assert np.linalg.norm(g - r) <= BF16_GRAD_REL * max(np.linalg.norm(r), 1e-30), k
    # and the bf16 run really differs from the fp32 engine (the flag reaches the kernels)
    model.train_bf16 = False
    _, p32 = _loss(model, torch.from_numpy(feats_np).to(gpu_device), torch.from_numpy(caps_np).to(gpu_device),
                   lengths)
    assert not torch.equal(p32[0].detach(), packed[0].detach())


def test_train_bf16_small_vocab_vs_fp32(gpu_device):
    """A vocabulary far below the channel count (100 < 2048) at a small batch: the bf16 step's packed
    W_a slot is sized for the larger of the two (the slot held only H x rup64(vocab)), so
    the encoder GEMM's operands are intact -- the bf16 step agrees with the fp32 step within the bf16
    tolerances, gradients included."""
    B, L = 4, 7
    lengths = [6, 5, 5, 3]
    cf = Config(vocab_length=100)
    rng = np.random.default_rng(2)
    caps = torch.from_numpy(rng.integers(0, 100, size=(B, L)).astype(np.int64)).to(gpu_device)
    caps[:, 0] = 1
    feats = torch.from_numpy(synth.make_features(B, seed=4)).to(gpu_device)
    out = {}
    for bf16 in (False, True):
        model = Encoder2Decoder(cf).to(gpu_device).load_synthetic(5, bias_noise=0.01)
        model.train_bf16 = bf16
        loss, packed = _loss(model, feats, caps, lengths)
        loss.backward()
        out[bf16] = (packed[0].detach().double(), loss.item(), {k: p.grad.detach().double() for k, p in model.named_parameters()})
    s32, l32, g32 = out[False]
    s16, l16, g16 = out[True]
    assert torch.linalg.norm(s16 - s32) <= BF16_SCORE_REL * torch.linalg.norm(s32)
    assert abs(l16 - l32) <= BF16_LOSS_REL * abs(l32)
    for k in g32:
        assert torch.linalg.norm(g16[k] - g32[k]) <= BF16_GRAD_REL * max(torch.linalg.norm(g32[k]).item(), 1e-30), k


def test_train_bf16_deterministic_and_reduces_loss(gpu_device):
    B, L = 8, 10
    lengths = [9, 8, 8, 6, 5, 5, 3, 2]
    rng = np.random.default_rng(11)
    caps = torch.from_numpy(rng.integers(0, 10123, size=(B, L)).astype(np.int64)).to(gpu_device)
    caps[:, 0] = 1
    feats = torch.from_numpy(synth.make_features(B, seed=3)).to(gpu_device)
    grads = []
    for _ in range(2):
        model = _model(gpu_device)
        model.train_bf16 = True
        loss, _ = _loss(model, feats, caps, lengths)
        loss.backward()
        grads.append({k: p.grad.clone() for k, p in model.named_parameters()})
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k
    model = _model(gpu_device)
    model.train_bf16 = True
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        loss, _ = _loss(model, feats, caps, lengths)
        losses.append(loss.item())
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.decoder.LSTM.parameters(), 5.0)
        opt.step()
    assert losses[-1] < losses[0]

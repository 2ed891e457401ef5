"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the reference goldens.

Tolerances (fp32 end to end on both sides; the two differ only in summation order and libm ulps):
* token ids: bit-identical (the north-star bar);
* logits: |GPU - oracle| <= 1e-4 (north-star), typically ~1e-6;
* alpha / beta / encoder outputs: <= 2e-5 absolute.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

from adaptive_amd import synth

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-4
ATT_TOL = 2e-5


def _model(seed=123, bias_noise=0.0, dev="cuda:0"):
    from adaptive_amd import Config, Encoder2Decoder
    m = Encoder2Decoder(Config()).to(dev)
    m.load_synthetic(seed, bias_noise=bias_noise)
    return m


def _oracle(seed=123, bias_noise=0.0):
    from oracle.adaptive_oracle import OracleModel
    return OracleModel(synth.make_weights(seed, bias_noise=bias_noise))


@pytest.fixture(scope="module")
def model(gpu_device):
    return _model()


@pytest.fixture(scope="module")
def oracle():
    return _oracle()


def test_synth_features_bit_exact(gpu_device):
    from adaptive_amd.adaptive_attention import synthetic_features
    for B, row0 in [(2, 0), (3, 5)]:
        g = synthetic_features(B, gpu_device, seed=0, row0=row0).cpu().numpy()
        c = synth.make_features(B, seed=0, row0=row0)
        assert np.array_equal(g.view(np.uint32), c.view(np.uint32))


def test_encoder_tail(model, oracle, gpu_device):
    B = 5
    feats = synth.make_features(B)
    V, v_g, (h0, c0), a_g, VWv = model._encode(torch.from_numpy(feats).to(gpu_device))
    rV, rvg, (rh0, rc0), ra_g = oracle.encoder(torch.from_numpy(feats))
    assert np.array_equal(a_g.cpu().numpy(), ra_g.numpy()), "avg-pool must be bit-exact (sequential fp32 sum)"
    np.testing.assert_allclose(V.cpu().numpy(), rV.numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(v_g.cpu().numpy(), rvg.numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(h0.cpu().numpy()[:, 0], rh0.numpy()[0], atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(c0.cpu().numpy()[:, 0], rc0.numpy()[0], atol=ATT_TOL, rtol=0)
    Wv = oracle.w["decoder.adaptive.atten.affine_v.weight"]
    ref_vwv = torch.nn.functional.linear(rV, Wv).numpy()
    got = VWv.cpu().numpy()
    np.testing.assert_allclose(got[..., :49], ref_vwv, atol=ATT_TOL, rtol=0)
    assert np.all(got[..., 49:] == 0)


@pytest.mark.parametrize("B", [67, 512])
def test_split_bf16_encoder_is_fp32_accurate(model, oracle, gpu_device, B):
    """The bf16x3 encoder (3-way bf16 split on bf16 MFMA: k_enc_v4 + k_gemm3 heads) vs an fp64
    reference: its error is of the same order as the fp32-MFMA encoder's (k_enc_v + k_enc_heads;
    K = 2048 fp32 accumulation), far below the 2e-5 parity tolerance.  B = 67 -> 3283 rows: a last
    two-image workgroup holding one image; B = 512: the bench grid."""
    feats = torch.from_numpy(synth.make_features(B, seed=3)).to(gpu_device)
    out4 = model._encode(feats)
    V4 = out4[0].cpu().numpy().astype(np.float64)
    try:
        model.fp32_encoder = True
        out1 = model._encode(feats)
        V1 = out1[0].cpu().numpy().astype(np.float64)
    finally:
        model.fp32_encoder = False
    A = feats.cpu().numpy().astype(np.float64).reshape(B, 2048, 49).transpose(0, 2, 1)
    W = oracle.w["encoder.affine_a.weight"].numpy().astype(np.float64)
    b = oracle.w["encoder.affine_a.bias"].numpy().astype(np.float64)
    pre = A @ W.T + b
    ref = np.maximum(pre, 0.0)
    scale = np.abs(A) @ np.abs(W).T + np.abs(b)          # sum_k |a_k w_k| + |b| per output
    e1 = np.abs(V1 - ref) / scale
    e4 = np.abs(V4 - ref) / scale
    assert e4.max() < 2e-6, e4.max()                     # fp32 GEMM class: ~K u / sqrt(K) << 1e-5
    assert e4.max() < 4 * e1.max() + 1e-7, (e4.max(), e1.max())
    assert np.abs(V4 - ref).max() < ATT_TOL / 2
    # heads: k_gemm3 (bf16x3, default) and k_enc_heads (fp32 MFMA) vs fp64
    a_g = out4[3].cpu().numpy().astype(np.float64)
    assert np.array_equal(out4[3].cpu().numpy(), out1[3].cpu().numpy()), "fused avg-pool == k_avgpool"
    for key, act, got4, got1 in (("encoder.affine_b", np.maximum, out4[1], out1[1]),
                                 ("encoder.affine_h0", np.tanh, out4[2][0][:, 0], out1[2][0][:, 0]),
                                 ("encoder.affine_c0", np.tanh, out4[2][1][:, 0], out1[2][1][:, 0])):
        Wh = oracle.w[key + ".weight"].numpy().astype(np.float64)
        bh = oracle.w[key + ".bias"].numpy().astype(np.float64)
        pre = a_g @ Wh.T + bh
        r = np.maximum(pre, 0.0) if act is np.maximum else np.tanh(pre)
        sc = np.abs(a_g) @ np.abs(Wh).T + np.abs(bh)
        e4 = np.abs(got4.cpu().numpy() - r) / sc
        e1 = np.abs(got1.cpu().numpy() - r) / sc
        assert e4.max() < 2e-6 and e4.max() < 4 * e1.max() + 1e-7, (key, e4.max(), e1.max())


def test_decode_step_logits(model, oracle, gpu_device):
    """One Decoder.forward step (T == 1) from the encoder states: logits within 1e-4."""
    B = 7
    feats = torch.from_numpy(synth.make_features(B, seed=3))
    rV, rvg, rstates, _ = oracle.encoder(feats)
    caps = torch.full((B, 1), 1, dtype=torch.int64)
    r_scores, r_alpha, r_beta, r_states = oracle.decoder(rV, rvg, caps, rstates)
    V, v_g, (h0, c0), _, _ = model._encode(feats.to(gpu_device))
    scores, alpha, beta, (h1, c1) = model.decoder(V, v_g, caps.to(gpu_device), (h0, c0))
    np.testing.assert_allclose(scores.cpu().numpy(), r_scores.numpy(), atol=LOGIT_TOL, rtol=0)
    np.testing.assert_allclose(alpha.cpu().numpy(), r_alpha.numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(beta.cpu().numpy(), r_beta.numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(h1.cpu().numpy(), r_states[0].numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(c1.cpu().numpy(), r_states[1].numpy(), atol=ATT_TOL, rtol=0)
    assert torch.equal(model._last_tokens.cpu(), r_scores.max(2)[1].reshape(B))
    # second step, fed the oracle's tokens
    caps2 = r_scores.max(2)[1]
    r2 = oracle.decoder(rV, rvg, caps2, r_states)
    s2 = model.decoder(V, v_g, caps2.to(gpu_device), (h1, c1))
    np.testing.assert_allclose(s2[0].cpu().numpy(), r2[0].numpy(), atol=LOGIT_TOL, rtol=0)


@pytest.mark.parametrize("case,seed,noise,fseed,B", [
    ("ref_b4", 123, 0.0, 0, 4),
    ("ref_b64", 123, 0.0, 0, 64),
    ("biased_b16", 99, 0.02, 5, 16),
])
def test_greedy_vs_reference_golden(case, seed, noise, fseed, B, gpu_device):
    g = load_golden(case)
    m = _model(seed, noise)
    feats = torch.from_numpy(synth.make_features(B, seed=fseed)).to(gpu_device)
    ids, alpha, beta = m.sampler(feats, max_len=20)
    ids = ids.cpu().numpy()
    assert ids.shape == (B, 20) and ids.dtype == np.int64
    mism = np.argwhere(ids != g["ids"])
    assert mism.size == 0, f"token mismatch at {mism[:5].tolist()} (margins {g['margin'][tuple(mism[0])] if mism.size else None})"
    if "alpha" in g:
        np.testing.assert_allclose(alpha.cpu().numpy(), g["alpha"], atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(beta.cpu().numpy(), g["beta"], atol=ATT_TOL, rtol=0)


def test_greedy_b512_vs_reference_golden(gpu_device):
    g = load_golden("ref_b512")
    m = _model()
    feats = torch.from_numpy(synth.make_features(512)).to(gpu_device)
    ids, alpha, beta = m.sampler(feats, max_len=20)
    ids = ids.cpu().numpy()
    mism = np.argwhere(ids != g["ids"])
    assert mism.size == 0, f"{len(mism)} token mismatches, first at {mism[:3].tolist()}, margin there {g['margin'][tuple(mism[0])]}"
    np.testing.assert_allclose(beta.cpu().numpy(), g["beta"], atol=ATT_TOL, rtol=0)
    # alpha of every 4th row (all eight 64-row tiles of the step kernels), pinned by the reference
    np.testing.assert_allclose(alpha.cpu().numpy()[::4], g["alpha_s4"], atol=ATT_TOL, rtol=0)


def test_batch_invariance(model, gpu_device):
    """Row i decoded inside B=300 equals row i decoded alone / inside a ragged batch, bitwise."""
    feats = torch.from_numpy(synth.make_features(300, seed=11)).to(gpu_device)
    ids, alpha, beta = model.sampler(feats, max_len=12)
    for lo, hi in [(0, 1), (37, 74), (250, 300)]:
        i2, a2, b2 = model.sampler(feats[lo:hi].contiguous(), max_len=12)
        assert torch.equal(i2, ids[lo:hi])
        assert torch.equal(a2, alpha[lo:hi])
        assert torch.equal(b2, beta[lo:hi])


@pytest.mark.parametrize("exact", [False, True])
def test_decode_plan_replay_equals_sampler(model, gpu_device, exact):
    """A DecodePlan (the whole decode captured once into a hipGraph over buffers the plan owns) gives
    sampler's results bit for bit, for every batch copied into it -- including batches held in
    freshly allocated tensors -- and keeps nothing of the caller's."""
    import weakref
    from adaptive_amd import DecodePlan
    B = 192
    plan = DecodePlan(model, B, max_len=7, exact_vocab=exact)
    for seed in (17, 18, 17):
        feats = torch.from_numpy(synth.make_features(B, seed=seed)).to(gpu_device)
        ref = model.sampler(feats, max_len=7, exact_vocab=exact)
        got = plan(feats)
        for r, g in zip(ref, got):
            assert torch.equal(r, g)
        w = weakref.ref(feats)
        del feats, got
        assert w() is None, "DecodePlan retained the caller's batch"
    plan.close()


@pytest.mark.parametrize("hidden,B", [(256, 37), (768, 20), (1024, 24)])
def test_other_hidden_sizes_vs_oracle(gpu_device, hidden, B):
    """The general-dims kernels: hidden 256 (k_vscreen2 tiles, k_enc_v4<2>), 768 and 1024 (the 64 x 64
    screen k_vscreen, the 128 x 128-tile encoder k_enc_v3, k_atten<HPT>) against the oracle; the
    screened ids equal the exact-vocab ids (the screen bound's H-dependent accumulation term,
    sc_acc(H))."""
    from adaptive_amd import Config, Encoder2Decoder
    from oracle.adaptive_oracle import OracleModel
    cf = Config(adaptive_word_embed_size=256, adaptive_lstm_hidden_size=hidden, vocab_length=3001)
    m = Encoder2Decoder(cf).to(gpu_device)
    m.load_synthetic(7)
    feats = synth.make_features(B, seed=29)
    ids, alpha, beta = m.sampler(torch.from_numpy(feats).to(gpu_device), max_len=12)
    r_ids, r_alpha, r_beta = OracleModel(synth.make_weights(7, m.dims)).sampler(torch.from_numpy(feats), max_len=12)
    assert torch.equal(ids.cpu(), r_ids)
    np.testing.assert_allclose(alpha.cpu().numpy(), r_alpha.numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(beta.cpu().numpy(), r_beta.numpy(), atol=ATT_TOL, rtol=0)
    ex = m.sampler(torch.from_numpy(feats).to(gpu_device), max_len=12, exact_vocab=True)
    assert torch.equal(ex[0].cpu(), r_ids)


def test_greedy_matches_oracle_odd_batch(model, oracle, gpu_device):
    B = 37
    feats = synth.make_features(B, seed=21)
    ids, alpha, beta = model.sampler(torch.from_numpy(feats).to(gpu_device), max_len=30)  # reference default
    r_ids, r_alpha, r_beta = oracle.sampler(torch.from_numpy(feats), max_len=30)
    assert torch.equal(ids.cpu(), r_ids)
    np.testing.assert_allclose(alpha.cpu().numpy(), r_alpha.numpy(), atol=ATT_TOL, rtol=0)
    np.testing.assert_allclose(beta.cpu().numpy(), r_beta.numpy(), atol=ATT_TOL, rtol=0)


def test_argmax_ties_pick_first_index(gpu_device):
    """Copy each step-0 winner's vocab row to one lower and one higher index: the logits tie
    exactly (same weights, same accumulation order), and the lower index must win, as torch's
    max(2)[1] returns the first maximal index (adaptive_attention.py:201)."""
    m = _model()
    feats = torch.from_numpy(synth.make_features(6, seed=2)).to(gpu_device)
    ids0, _, _ = m.sampler(feats, max_len=1)
    winners = sorted(set(ids0[:, 0].tolist()))
    used = set(winners)
    low, high = {}, {}
    for tok in winners:
        lo = next(i for i in range(tok - 1, -1, -1) if i not in used) if tok > 0 else None
        hi = next(i for i in range(tok + 1, 10123) if i not in used)
        used.update(x for x in (lo, hi) if x is not None)
        low[tok], high[tok] = lo, hi
    with torch.no_grad():
        W = m.decoder.adaptive.mlp.weight
        b = m.decoder.adaptive.mlp.bias
        for tok in winners:
            for dst in (low[tok], high[tok]):
                if dst is not None:
                    W[dst].copy_(W[tok])
                    b[dst].copy_(b[tok])
    ids1, _, _ = m.sampler(feats, max_len=1)
    for b_, tok in enumerate(ids0[:, 0].tolist()):
        want = low[tok] if low[tok] is not None else tok
        assert ids1[b_, 0].item() == want


def test_edge_shapes(model, gpu_device):
    feats = torch.from_numpy(synth.make_features(3)).to(gpu_device)
    ids, alpha, beta = model.sampler(feats[:0], max_len=20)
    assert ids.shape == (0, 20) and alpha.shape == (0, 20, 49) and beta.shape == (0, 20, 1)
    ids, alpha, beta = model.sampler(feats, max_len=0)
    assert ids.shape == (3, 0)
    i1, _, _ = model.sampler(feats, max_len=1)
    i5, _, _ = model.sampler(feats, max_len=5)
    assert torch.equal(i1, i5[:, :1])


def test_errors_are_loud(model, gpu_device):
    with pytest.raises(ValueError):
        model.sampler(torch.zeros(2, 2048, 7, 6, device=gpu_device))
    with pytest.raises(RuntimeError):
        model.sampler(torch.zeros(2, 2048, 7, 7))
    with pytest.raises(IndexError):
        V, v_g, st, _, _ = model._encode(torch.from_numpy(synth.make_features(2)).to(gpu_device))
        model.decoder(V, v_g, torch.full((2, 1), 10123, dtype=torch.int64, device=gpu_device), st)


def test_rescoring_logits_bit_identical_to_fp32_gemm(model, gpu_device):
    """The exact-fp32 rescoring (used after the bf16 screen) reproduces the fp32 MFMA GEMM's logits
    bit for bit (same fma order), so screening never changes which column wins a near-tie."""
    g = torch.Generator().manual_seed(0)
    u = (torch.rand(77, 512, generator=g) * 2 - 1).to(gpu_device)
    full = model.vocab_logits(u)
    cols = torch.randint(0, 10123, (77, 300), generator=g).to(gpu_device)
    cols[:, 0] = 10122
    cols[:, 1] = 0
    part = model.vocab_logits(u, cols)
    assert torch.equal(part, torch.gather(full, 1, cols.long()))
    ref = u.cpu() @ model.decoder.adaptive.mlp.weight.detach().cpu().T + model.decoder.adaptive.mlp.bias.detach().cpu()
    np.testing.assert_allclose(full.cpu().numpy(), ref.numpy(), atol=1e-4, rtol=0)


@pytest.mark.parametrize("seed,noise,fseed,B,T", [(123, 0.0, 0, 512, 20), (99, 0.02, 7, 300, 20), (5, 0.0, 3, 64, 30)])
def test_screened_vocab_equals_exact_vocab(seed, noise, fseed, B, T, gpu_device):
    """bf16 screen + exact rescoring == full fp32 logits argmax, token for token."""
    m = _model(seed, noise)
    feats = torch.from_numpy(synth.make_features(B, seed=fseed)).to(gpu_device)
    a = m.sampler(feats, max_len=T)
    b = m.sampler(feats, max_len=T, exact_vocab=True)
    assert torch.equal(a[0], b[0])
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


@pytest.mark.parametrize("B,T", [(512, 20), (300, 9), (67, 5), (1, 4), (3, 2), (130, 1)])
def test_fused_rescoring_equals_split(B, T, gpu_device):
    """Step t-1's rescoring inside step t's LSTM launch (the default) == its own launch per step
    (AA_DECODE_SPLIT_RESCORE) == the LSTM workgroups rescoring every unpublished row themselves
    (AA_DECODE_RS_SELF, the no-wait fallback that keeps the fused launch deadlock-free) == the screen on
    four waves per tile (AA_DECODE_SCREEN4, k_vscreen2 instead of k_vscreen8): ids, alpha and beta bit
    for bit, on odd and single-row batches and T = 1 (no fused launch)."""
    from adaptive_amd import _lib
    m = _model(99, 0.02)
    feats = torch.from_numpy(synth.make_features(B, seed=B + T)).to(gpu_device)
    a = m.sampler(feats, max_len=T)
    for extra in (_lib.DECODE_SPLIT_RESCORE, _lib.DECODE_RS_SELF, _lib.DECODE_SCREEN4):
        m.decode_extra_flags = extra
        b = m.sampler(feats, max_len=T)
        m.decode_extra_flags = 0
        for x, y in zip(a, b):
            assert torch.equal(x, y), extra
    ex = m.sampler(feats, max_len=T, exact_vocab=True)
    assert torch.equal(ex[0], a[0])


def test_fused_rescoring_nan_vocab_weights(gpu_device):
    """An all-NaN vocabulary projection leaves the screen's summaries NaN and the candidate lists
    empty: the rescoring then scores every column and still publishes a non-zero key, so the fused
    launch's GEMM workgroups find every key published (no 50 us bounded poll per step) and the three
    launch structures agree bit for bit."""
    from adaptive_amd import _lib
    m = _model(5, 0.02)
    with torch.no_grad():
        m.decoder.adaptive.mlp.weight.fill_(float("nan"))
    feats = torch.from_numpy(synth.make_features(67, seed=8)).to(gpu_device)
    a = m.sampler(feats, max_len=4)
    assert bool(((a[0] >= 0) & (a[0] < m.dims.vocab)).all())
    for extra in (_lib.DECODE_SPLIT_RESCORE, _lib.DECODE_RS_SELF, _lib.DECODE_SCREEN4):
        m.decode_extra_flags = extra
        b = m.sampler(feats, max_len=4)
        m.decode_extra_flags = 0
        for x, y in zip(a, b):
            assert torch.equal(x, y), extra


def test_all_columns_tied_rescore_overflow(gpu_device):
    """W_m = 0, b_m = 0: every logit is exactly 0, so every column is a candidate (k_vrescore's
    candidate list overflows into its all-columns fallback).  The first index (0) must win
    everywhere, as torch's max(2)[1]."""
    m = _model()
    with torch.no_grad():
        m.decoder.adaptive.mlp.weight.zero_()
        m.decoder.adaptive.mlp.bias.zero_()
    feats = torch.from_numpy(synth.make_features(130, seed=4)).to(gpu_device)
    ids, _, _ = m.sampler(feats, max_len=3)
    assert torch.equal(ids, torch.zeros_like(ids))
    ex, _, _ = m.sampler(feats, max_len=3, exact_vocab=True)
    assert torch.equal(ex, ids)

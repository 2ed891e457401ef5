"""CPU: the oracle restatement against golden vectors produced by the REAL reference sampler
(tests/golden/make_golden.py imported code_src/models/adaptive_attention.py in the build container).
This is what pins the oracle; the GPU tests then compare the HIP path with the oracle."""
import numpy as np
import pytest
import torch

from conftest import load_golden

from adaptive_amd import synth
from oracle.adaptive_oracle import OracleModel, top2_margin

CASES = {"ref_b4": (123, 0.0, 0, 4), "biased_b16": (99, 0.02, 5, 16), "ref_b64": (123, 0.0, 0, 64)}


@pytest.mark.parametrize("case", list(CASES))
def test_oracle_matches_reference_golden(case, manifest):
    seed, noise, fseed, B = CASES[case]
    g = load_golden(case)
    state = synth.make_weights(seed, bias_noise=noise)
    assert synth.digest(state) == manifest["cases"][case]["weights_sha256"]
    feats = synth.make_features(B, seed=fseed)
    assert synth.digest({"f": feats})["f"] == manifest["cases"][case]["features_sha256"]
    ids, alpha, beta, scores = OracleModel(state).sampler(torch.from_numpy(feats), max_len=20, keep_scores=True)
    assert np.array_equal(ids.numpy(), g["ids"].astype(np.int64))
    np.testing.assert_allclose(beta.numpy(), g["beta"], atol=1e-6, rtol=0)
    if "alpha" in g:
        np.testing.assert_allclose(alpha.numpy(), g["alpha"], atol=1e-6, rtol=0)
    if "scores_t0" in g:
        np.testing.assert_allclose(scores[:, 0].numpy(), g["scores_t0"], atol=1e-5, rtol=0)
        np.testing.assert_allclose(scores[:2, :2].numpy(), g["scores_r01_t01"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(top2_margin(scores).numpy(), g["margin"], atol=1e-5, rtol=0)


def test_oracle_b512_ids_match_reference_golden():
    g = load_golden("ref_b512")
    feats = synth.make_features(512)
    ids, alpha, beta = OracleModel(synth.make_weights(123)).sampler(torch.from_numpy(feats), max_len=20)
    assert np.array_equal(ids.numpy(), g["ids"].astype(np.int64))
    np.testing.assert_allclose(beta.numpy(), g["beta"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(alpha.numpy()[::4], g["alpha_s4"], atol=1e-6, rtol=0)  # every 4th row


def test_oracle_row_independence():
    """Rows decode independently: a row alone == the same row inside a batch."""
    feats = synth.make_features(12, seed=4)
    m = OracleModel(synth.make_weights(123))
    ids, _, _ = m.sampler(torch.from_numpy(feats), max_len=10)
    for i in (0, 5, 11):
        one, _, _ = m.sampler(torch.from_numpy(feats[i:i + 1]), max_len=10)
        assert torch.equal(one[0], ids[i])


def test_reference_defect_d1_shape_semantics():
    """The oracle keeps the baseline transpose (baseline_attention.py:251-252): states [1,B,H]."""
    m = OracleModel(synth.make_weights(123))
    V, v_g, (h, c), a_g = m.encoder(torch.from_numpy(synth.make_features(3)))
    assert h.shape == (1, 3, 512) and c.shape == (1, 3, 512) and V.shape == (3, 49, 512) and a_g.shape == (3, 2048)


def test_train_oracle_matches_reference_golden():
    """TrainOracle (teacher-forced forward + CE + autograd) against the real reference's packed
    scores, loss and gradients (tests/golden/train_b4.npz, make_golden_train.py)."""
    from oracle.adaptive_oracle import TrainOracle
    g = load_golden("train_b4")
    m = TrainOracle(synth.make_weights(123, bias_noise=0.02))
    feats = torch.from_numpy(synth.make_features(4, seed=7))
    caps = torch.from_numpy(g["captions"])
    loss, packed = m.loss(feats, caps, g["lengths"].tolist())
    assert packed[1].tolist() == g["batch_sizes"].tolist()
    np.testing.assert_allclose(packed[0].detach().numpy(), g["scores"], atol=1e-5, rtol=0)
    assert abs(loss.item() - float(g["loss"])) <= 1e-6 * abs(float(g["loss"]))
    loss.backward()
    for k, p in m.w.items():
        got = p.grad.detach().numpy().reshape(-1).astype(np.float64)
        idx = g["g:" + k + ":idx"] if "g:" + k + ":idx" in g else slice(None)
        ref = np.asarray(g["g:" + k], np.float64)
        assert np.abs(got[idx] - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-30), k

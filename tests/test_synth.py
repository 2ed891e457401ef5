"""CPU: the counter-based generator is deterministic, shard-consistent and has the init statistics."""
import math

import numpy as np

from adaptive_amd import synth


def test_known_answers():
    # splitmix64 reference values (seed 0 stream): first outputs of the published algorithm
    assert synth._mix_int(0x9E3779B97F4A7C15) == 0xE220A8397B1DCDAF
    u = synth.uniform24(0, 0, 3)
    assert np.array_equal(u, np.array([0xE220A8 / 2 ** 24, 0x6E789E / 2 ** 24, 0x06C45D / 2 ** 24]))


def test_features_shard_consistent():
    full = synth.make_features(6, seed=0)
    part = synth.make_features(2, seed=0, row0=3)
    assert np.array_equal(full[3:5], part)
    assert full.dtype == np.float32 and full.min() >= 0 and full.max() < 1


def test_weights_deterministic_and_distributions():
    a = synth.make_weights(123)
    b = synth.make_weights(123)
    assert synth.digest(a) == synth.digest(b)
    c = synth.make_weights(124)
    assert synth.digest(a)["decoder.adaptive.mlp.weight"] != synth.digest(c)["decoder.adaptive.mlp.weight"]
    mlp = a["decoder.adaptive.mlp.weight"]
    assert abs(mlp.std() - math.sqrt(2 / 512)) / math.sqrt(2 / 512) < 0.01
    emb = a["decoder.embed.weight"]
    assert abs(emb.std() - 1.0) < 0.01 and abs(emb.mean()) < 0.01
    b_ih = a["decoder.LSTM.bias_ih_l0"]
    assert np.all(b_ih[512:1024] == 0.5) and np.all(b_ih[:512] == 0) and np.all(b_ih[1024:] == 0)
    wa = a["encoder.affine_a.weight"]
    assert np.abs(wa).max() <= math.sqrt(6 / 2048)


def test_bias_noise_only_touches_biases():
    a = synth.make_weights(5)
    b = synth.make_weights(5, bias_noise=0.02)
    for k in a:
        same = np.array_equal(a[k], b[k])
        assert same == (not k.rsplit(".", 1)[-1].startswith("bias")), k

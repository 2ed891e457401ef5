"""GPU: sampler() under the reference's own evaluation loop (code_src/tools/utils.py:23-29,167-171):
every call gets a FRESHLY allocated batch (``images = to_var(images)`` -> ``.cuda()``; with the trunk,
``features()`` also returns a fresh tensor per call), so the caching allocator keeps handing the
decode the block the previous batch freed.  sampler() must not capture or cache anything per input
pointer, must not retain the caller's tensors, and must return the same ids as for a resident batch.
"""
import gc
import weakref

import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder, synth
from adaptive_amd.adaptive_attention import synthetic_features

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(gpu_device):
    return Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)


def test_fresh_batch_per_call(model, gpu_device):
    B, T = 256, 20
    srcs = [synthetic_features(B, gpu_device, seed=s) for s in (3, 4)]
    ref = [model.sampler(x, max_len=T) for x in srcs]
    captures0 = Encoder2Decoder._captures
    seen = set()
    for i in range(8):
        x = torch.empty_like(srcs[0])   # fresh allocation, as to_var(images).cuda() per batch
        x.copy_(srcs[i % 2])
        seen.add(x.data_ptr())
        w = weakref.ref(x)
        ids, alpha, beta = model.sampler(x, max_len=T)
        del x
        gc.collect()
        assert w() is None, "sampler retained the caller's batch"
        assert torch.equal(ids, ref[i % 2][0])
        assert torch.equal(alpha, ref[i % 2][1]) and torch.equal(beta, ref[i % 2][2])
    assert Encoder2Decoder._captures == captures0, "sampler captured a graph"
    assert len(seen) <= 2  # the allocator did hand back the freed block (the pattern under test)


def test_fresh_images_per_call_with_trunk(gpu_device):
    """trunk=True: images [B,3,224,224] in fresh tensors each call -> features() -> sampler."""
    m = Encoder2Decoder(Config(), trunk=True).to(gpu_device).load_synthetic(123).eval()
    g = torch.Generator().manual_seed(0)
    imgs = [torch.rand(6, 3, 224, 224, generator=g) for _ in range(2)]
    with torch.no_grad():
        # one untimed call first: MIOpen may pick the trunk's convolution algorithms on the first call
        # of a shape and switch to the tuned ones after it (different rounding in the random-init
        # trunk's features: the alphas moved by up to 2e-2 between those calls on one box)
        for im in imgs:
            m.sampler(im.to(gpu_device), max_len=8)
        ref = [m.sampler(im.to(gpu_device), max_len=8) for im in imgs]
    captures0 = Encoder2Decoder._captures
    for i in range(8):
        x = imgs[i % 2].to(gpu_device)  # a new device tensor per call, as utils.py:23-29
        w = weakref.ref(x)
        with torch.no_grad():
            ids, alpha, beta = m.sampler(x, max_len=8)
        del x
        gc.collect()
        assert w() is None
        assert torch.equal(ids, ref[i % 2][0]) and torch.equal(alpha, ref[i % 2][1])
    assert Encoder2Decoder._captures == captures0


def test_features_fresh_tensor_equals_resident(model, gpu_device):
    """The same batch through a fresh buffer and through a resident one: identical results, and the
    results do not alias the input (the caller may free it at once)."""
    feats = torch.from_numpy(synth.make_features(64, seed=5)).to(gpu_device)
    a = model.sampler(feats, max_len=12)
    b = model.sampler(feats.clone(), max_len=12)
    for x, y in zip(a, b):
        assert torch.equal(x, y)

"""GPU: DecodePipeline (several batches in flight on their own HIP streams) returns exactly what
one sampler() call per batch returns, in submission order, for fresh inputs (direct launches) and
for a repeated input (captured decode plans)."""
import pytest
import torch

from adaptive_amd import Config, Encoder2Decoder
from adaptive_amd.adaptive_attention import synthetic_features
from adaptive_amd.pipeline import DecodePipeline

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model(gpu_device):
    return Encoder2Decoder(Config()).to(gpu_device).load_synthetic(123)


@pytest.mark.parametrize("depth", [1, 2, 3, 4])
def test_pipeline_equals_sequential(model, gpu_device, depth):
    batches = [synthetic_features(B, gpu_device, seed=s) for s, B in ((1, 64), (2, 100), (3, 64), (4, 7), (5, 128))]
    ref = [model.sampler(f, max_len=12, graph=False) for f in batches]
    got = list(DecodePipeline(model, max_len=12, depth=depth).run(iter(batches)))
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        for a, b in zip(g, r):
            assert torch.equal(a, b)


@pytest.mark.parametrize("depth", [2, 4])
def test_pipeline_repeated_input_uses_plans(model, gpu_device, depth):
    """bench.py's headline region: the same resident batch through `depth` slots, replayed plans."""
    f = synthetic_features(512, gpu_device, seed=9)
    ref = model.sampler(f, max_len=20, graph=False)
    pipe = DecodePipeline(model, max_len=20, depth=depth, graph=True)
    outs = list(pipe.run([f] * (3 * depth + 1)))
    assert any(len(s.plans) for s in pipe._slots)
    for out in outs:
        for a, b in zip(out, ref):
            assert torch.equal(a, b)

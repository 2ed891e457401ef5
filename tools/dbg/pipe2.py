import sys, time, itertools, torch
sys.path.insert(0, '.')
from adaptive_amd import Config, Encoder2Decoder, _lib
from adaptive_amd.adaptive_attention import synthetic_features
from adaptive_amd.pipeline import DecodePipeline
dev = torch.device('cuda', 0)
m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
B, T = 512, 20
feats = synthetic_features(B, dev, seed=0)
graph = sys.argv[1] == 'graph'
m.sampler(feats, max_len=T); m.sampler(feats, max_len=T); m.sampler(feats, max_len=T)  # a model plan too, as in bench.py
for depth in (1, 2, 3):
    pipe = DecodePipeline(m, max_len=T, depth=depth, graph=graph)
    for _ in pipe.run(itertools.repeat(feats, 2 * depth + 1)):
        pass
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for out in pipe.run(itertools.repeat(feats, 30)):
            n += 1
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{sys.argv[1]} depth {depth}: {(t2 - t0) / 30 * 1e3:.3f} ms/batch (host loop {(t1 - t0) / 30 * 1e3:.3f} ms/batch)", flush=True)

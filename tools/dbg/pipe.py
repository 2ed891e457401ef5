import sys, time, torch
sys.path.insert(0, '.')
from adaptive_amd import Config, Encoder2Decoder, _lib
from adaptive_amd.adaptive_attention import synthetic_features, _Plan
dev = torch.device('cuda', 0)
m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
B, T = 512, 20
feats = synthetic_features(B, dev, seed=0)
lib = _lib.load(); model = m._model_struct()
plans = [_Plan(lib, model, feats, B, T, 0, 1, m._c_dims(), dev) for _ in range(3)]
streams = [torch.cuda.Stream(dev) for _ in range(3)]
def run(nst, K=60):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        j = i % nst
        _lib.check(lib.aa_decode_plan_launch(plans[j].handle, streams[j].cuda_stream), "launch")
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K
for nst in (1, 2, 3, 1, 2, 3):
    ms = run(nst) * 1e3
    print(f"streams {nst}: {ms:.3f} ms/batch  {B / ms * 1e3:.0f} captions/s", flush=True)
ref = plans[0].ids.clone()
print("same ids", all(torch.equal(p.ids, ref) for p in plans))

"""Probe the GPU box's CPU share: affinity, cgroup quota, and the oracle sampler's time per thread count."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from adaptive_amd import synth
from oracle.adaptive_oracle import OracleModel
print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count(), flush=True)
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    try:
        print(p, open(p).read().strip(), flush=True)
    except Exception as e:
        print(p, "n/a", flush=True)
m = OracleModel(synth.make_weights(123))
f = torch.from_numpy(synth.make_features(64, seed=0))
for th in [int(x) for x in sys.argv[1:]]:
    torch.set_num_threads(th)
    m.sampler(f[:4], max_len=2)
    t = time.perf_counter(); m.sampler(f, max_len=5); el = time.perf_counter() - t
    print(f"threads {th}: B=64 T=5 {el:.3f} s", flush=True)

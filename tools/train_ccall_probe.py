"""How much of a training step's host time is spent inside the C calls (kernel launches) vs around
them in Python / autograd (tools only; round 6).  Wraps the ctypes entry points of one library
instance with perf_counter timers and runs bench_train's step.

    python tools/train_ccall_probe.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench_train import make_batch, step  # noqa: E402
from adaptive_amd import Config, Encoder2Decoder, _lib  # noqa: E402
from adaptive_amd import optim as aa_optim  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402

NAMES = ("aa_train_forward_aux", "aa_train_backward_aux", "aa_cross_entropy_forward", "aa_cross_entropy_backward",
         "aa_adam_step", "aa_clip_grad_norm", "aa_train_workspace_bytes")


class Timed:
    def __init__(self, fn):
        self.fn, self.t, self.n = fn, 0.0, 0

    def __call__(self, *a):
        t0 = time.perf_counter()
        r = self.fn(*a)
        self.t += time.perf_counter() - t0
        self.n += 1
        return r


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    timers = {}
    for n in NAMES:
        timers[n] = Timed(getattr(lib, n))
        setattr(lib, n, timers[n])
    caps_np, lengths = make_batch(128, 18)
    model = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    model.train_bf16 = True
    feats = synthetic_features(128, dev, seed=0)
    caps = torch.from_numpy(caps_np).to(dev)
    opt = aa_optim.Adam(model.parameters(), lr=1e-4)
    crit = aa_optim.CrossEntropyLoss()
    for _ in range(10):
        step(model, opt, crit, feats, caps, lengths, aa_optim.clip_grad_norm_)
    torch.cuda.synchronize()
    for t in timers.values():
        t.t, t.n = 0.0, 0
    n = 40
    t0 = time.perf_counter()
    for _ in range(n):
        step(model, opt, crit, feats, caps, lengths, aa_optim.clip_grad_norm_)
    host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    print(f"per step: host loop {host * 1e3:.3f} ms, wall {wall * 1e3:.3f} ms")
    for k, t in timers.items():
        if t.n:
            print(f"  {k:28s} {t.t / n * 1e3:7.3f} ms per step ({t.n / n:.0f} calls)")


if __name__ == "__main__":
    main()

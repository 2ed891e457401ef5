"""Host-side profile of bench_train's step (tools only): cProfile over 40 steady-state steps, the
top entries by own time (ctypes calls into libadaptive_amd appear as their own rows).

    python tools/train_cprofile.py
"""
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench_train import make_batch, step  # noqa: E402
from adaptive_amd import Config, Encoder2Decoder  # noqa: E402
from adaptive_amd import optim as aa_optim  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    caps_np, lengths = make_batch(128, 18)
    model = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    model.train_bf16 = True
    feats = synthetic_features(128, dev, seed=0)
    caps = torch.from_numpy(caps_np).to(dev)
    opt = aa_optim.Adam(model.parameters(), lr=1e-4)
    crit = aa_optim.CrossEntropyLoss()
    for _ in range(6):
        step(model, opt, crit, feats, caps, lengths, aa_optim.clip_grad_norm_)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(40):
        step(model, opt, crit, feats, caps, lengths, aa_optim.clip_grad_norm_)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(28)


if __name__ == "__main__":
    main()

"""Measured errors of the config-5 training step (B = 128, T = 18) against the CPU oracle's autograd,
bf16 and fp32 GEMMs: the figures the tolerances in tests/test_gpu_configs.py and
tests/test_gpu_train.py are set from (tools only; GPU).

    python tools/train_tolerances.py > profiles/r05_train_tolerances.txt
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from adaptive_amd import Config, Encoder2Decoder, synth  # noqa: E402
from test_gpu_configs import _config5_batch, _gpu_loss  # noqa: E402


def main():
    from oracle.adaptive_oracle import TrainOracle
    dev = torch.device("cuda", 0)
    caps, lengths = _config5_batch()
    state = synth.make_weights(123, bias_noise=0.02)
    feats = synth.make_features(128, seed=0)
    oracle = TrainOracle(state)
    loss, packed = oracle.loss(torch.from_numpy(feats), torch.from_numpy(caps), lengths)
    loss.backward()
    rscores = packed[0].detach().double().numpy()
    rgrads = {k: v.grad.detach().double().numpy() for k, v in oracle.w.items()}
    for bf16 in (True, False):
        m = Encoder2Decoder(Config()).to(dev).load_synthetic(123, bias_noise=0.02)
        m.train_bf16 = bf16
        l, p = _gpu_loss(m, torch.from_numpy(feats).to(dev), torch.from_numpy(caps).to(dev), lengths)
        got = p[0].detach().cpu().double().numpy()
        l.backward()
        print(f"bf16={bf16}: scores rel-Frobenius {np.linalg.norm(got - rscores) / np.linalg.norm(rscores):.3e}, "
              f"max abs {np.abs(got - rscores).max():.3e}; loss rel {abs(l.item() - loss.item()) / abs(loss.item()):.3e}")
        worst = (0.0, "")
        for k, prm in m.named_parameters():
            g, r = prm.grad.detach().cpu().double().numpy(), rgrads[k]
            rel = np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)
            ent = np.abs(g - r).max() / max(np.abs(r).max(), 1e-30)
            print(f"   {k:48s} rel-Frobenius {rel:.3e}  max-entry/max {ent:.3e}")
            worst = max(worst, (rel, k))
        print(f"   worst gradient rel-Frobenius {worst[0]:.3e} ({worst[1]})")


if __name__ == "__main__":
    main()

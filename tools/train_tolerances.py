"""Measured errors of the config-5 training step (B = 128, T = 18) against the CPU oracle's autograd,
bf16 and fp32 GEMMs; of the train.py closure (three zero_grad / forward / CE / backward / clip /
Adam steps, bf16 GEMMs) against the same closure on the oracle; and of decoder(...) on whole
captions (T = 12) against the oracle's Decoder.forward: the figures the tolerances in
tests/test_gpu_configs.py and tests/test_gpu_train.py are set from (tools only; GPU).

    python tools/train_tolerances.py > profiles/r06_tolerances.txt
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
    closure(dev, caps, lengths, feats)
    decoder_whole_captions(dev)


def closure(dev, caps, lengths, feats):
    """test_config5_adam_clip_closure_vs_oracle's three steps: per-step loss and clip-norm errors."""
    from oracle.adaptive_oracle import TrainOracle
    oracle = TrainOracle(synth.make_weights(123, bias_noise=0.02))
    o_opt = torch.optim.Adam(list(oracle.w.values()), lr=1e-3)
    o_lstm = [oracle.w["decoder.LSTM." + n] for n in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    model = Encoder2Decoder(Config()).to(dev).load_synthetic(123, bias_noise=0.02)
    model.train_bf16 = True
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    f, c = torch.from_numpy(feats).to(dev), torch.from_numpy(caps).to(dev)
    of, oc = torch.from_numpy(feats), torch.from_numpy(caps)
    for i in range(3):
        model.zero_grad()
        opt.zero_grad()
        loss, _ = _gpu_loss(model, f, c, lengths)
        loss.backward()
        norm = torch.nn.utils.clip_grad_norm_(model.decoder.LSTM.parameters(), 5.0)
        opt.step()
        o_opt.zero_grad()
        rloss, _ = oracle.loss(of, oc, lengths)
        rloss.backward()
        rnorm = torch.nn.utils.clip_grad_norm_(o_lstm, 5.0)
        o_opt.step()
        print(f"closure step {i}: loss rel {abs(loss.item() - rloss.item()) / abs(rloss.item()):.3e}, "
              f"clip-norm rel {abs(norm.item() - rnorm.item()) / rnorm.item():.3e}")


def decoder_whole_captions(dev):
    """test_decoder_whole_captions_vs_oracle: max abs errors of scores, alpha, beta, h, c."""
    from oracle.adaptive_oracle import OracleModel
    B, T = 9, 12
    m = Encoder2Decoder(Config()).to(dev).load_synthetic(31, bias_noise=0.01)
    feats = torch.from_numpy(synth.make_features(B, seed=5)).to(dev)
    V, v_g, (h0, c0) = m.encoder(feats)
    rng = np.random.default_rng(3)
    caps = torch.from_numpy(rng.integers(0, 10123, size=(B, T)).astype(np.int64))
    caps[:, 0] = 1
    states = (h0.transpose(0, 1), c0.transpose(0, 1))
    sc, al, be, (h, c) = m.decoder(V, v_g, caps.to(dev), states)
    o = OracleModel(synth.make_weights(31, bias_noise=0.01))
    with torch.no_grad():
        osc, oal, obe, (oh, oc) = o.decoder(V.cpu(), v_g.cpu(), caps, (states[0].cpu().contiguous(),
                                                                     states[1].cpu().contiguous()))
    for name, x, y in (("scores", sc, osc), ("alpha", al, oal), ("beta", be, obe), ("h", h, oh), ("c", c, oc)):
        print(f"decoder T={T}: {name} max abs {float((x.cpu() - y).abs().max()):.3e}")


if __name__ == "__main__":
    main()

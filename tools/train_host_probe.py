"""Where does a training step's time go: host issue or GPU execution? (tools only)

The steady-state step time, the host time per phase, and one isolated step (queue idle before it)
split into the host's issue time and the GPU tail after the host is done; plus the step with the
packed targets computed once outside the loop.  (profiles/r05_train_host_probe.txt also holds a
"graphs=1" run of a since-removed step-graph cache that replayed each training call as a hipGraph.)

    python tools/train_host_probe.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench_train import make_batch  # noqa: E402
from adaptive_amd import Config, Encoder2Decoder  # noqa: E402
from adaptive_amd import optim as aa_optim  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402
from torch.nn.utils.rnn import pack_padded_sequence  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, T = 128, 18
    caps_np, lengths = make_batch(B, T)
    model = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    model.train_bf16 = True
    feats = synthetic_features(B, dev, seed=0)
    caps = torch.from_numpy(caps_np).to(dev)
    opt = aa_optim.Adam(model.parameters(), lr=1e-4)
    crit = aa_optim.CrossEntropyLoss()
    fixed_targets = pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0]

    def step(ph=None, pre=False):
        a = time.perf_counter()
        targets = fixed_targets if pre else pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0]
        b = time.perf_counter()
        model.zero_grad()
        opt.zero_grad()
        c = time.perf_counter()
        packed = model(feats, caps, lengths)
        d = time.perf_counter()
        loss = crit(packed[0], targets)
        e = time.perf_counter()
        loss.backward()
        f = time.perf_counter()
        aa_optim.clip_grad_norm_(model.decoder.LSTM.parameters(), 5.0)
        g = time.perf_counter()
        opt.step()
        h = time.perf_counter()
        if ph is not None:
            for k, x, y in (("targets", a, b), ("zero_grad", b, c), ("forward", c, d), ("loss", d, e),
                            ("backward", e, f), ("clip", f, g), ("adam", g, h)):
                ph[k] = ph.get(k, 0.0) + (y - x) * 1e3

    n = 40
    for mode in (0,):
        for _ in range(6):
            step()
        torch.cuda.synchronize()
        for pre in (False, True):
            t0 = time.perf_counter()
            for _ in range(n):
                step(pre=pre)
            torch.cuda.synchronize()
            print(f"graphs={mode} targets {'precomputed' if pre else 'per step '}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms/step")
        ph = {}
        torch.cuda.synchronize()
        for _ in range(n):
            step(ph)
        torch.cuda.synchronize()
        print(f"graphs={mode} host ms per phase:", {k: round(v / n, 3) for k, v in ph.items()},
              "sum", round(sum(ph.values()) / n, 3))
        iss, tail = [], []
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            iss.append((t1 - t0) * 1e3)
            tail.append((t2 - t1) * 1e3)
        iss.sort()
        tail.sort()
        print(f"graphs={mode} isolated step: host issue {iss[5]:.3f} ms, GPU tail after issue {tail[5]:.3f} ms "
              f"(total {iss[5] + tail[5]:.3f})")


if __name__ == "__main__":
    main()

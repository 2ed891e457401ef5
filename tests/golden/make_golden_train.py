"""Golden vectors for the teacher-forced training step, from the REAL reference on CPU.

Run in the survey/build container only:  python tests/golden/make_golden_train.py

Drives ``Encoder2Decoder.forward(images, captions, lengths)`` (``baseline_attention.py:206-230``,
inherited by ``adaptive_attention.Encoder2Decoder``) and the training closure's loss
(``train.py:63,204-210``: ``CrossEntropyLoss(packed_scores[0], targets)`` with
``targets = pack_padded_sequence(captions[:, 1:], lengths)``), then ``loss.backward()``.
Same stubs as make_golden.py (torchvision absent, trunk = identity on post-trunk features).
Defect D2 (the in-place ``states[i].transpose_(0, 1)`` of a view of a tanh output
makes backward raise on torch 2.10): the encoder returns clones of (h0, c0), as prescribed there.

Recorded: packed scores, loss, and for every parameter its gradient -- in full when it has at
most 65,536 elements, otherwise 4,096 entries at seeded random flat indices plus the norm.
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.nn.utils.rnn import pack_padded_sequence  # noqa: E402

from adaptive_amd import synth  # noqa: E402
from make_golden import Cf, load_reference  # noqa: E402

FULL_MAX = 65536
NSAMPLE = 4096


def train_case():
    """B = 4, captions of 7 tokens (<start> = 1 first), lengths 6, 5, 5, 3 (cap_len - 1, sorted)."""
    B, L = 4, 7
    lengths = [6, 5, 5, 3]
    rng = np.random.default_rng(2024)
    caps = rng.integers(2, 10123, size=(B, L)).astype(np.int64)
    caps[:, 0] = 1
    for b, n in enumerate(lengths):
        caps[b, n + 1:] = 0  # padding after the last token (never read by the packed loss)
    return caps, lengths


def main():
    torch.set_num_threads(8)
    aa = load_reference()
    state = synth.make_weights(123, bias_noise=0.02)
    feats = synth.make_features(4, seed=7)
    caps, lengths = train_case()
    torch.manual_seed(0)
    m = aa.Encoder2Decoder(Cf())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()}, strict=True)
    m.train()
    enc_forward = m.encoder.forward

    def enc_d2(images):  # D2: return clones so the in-place transpose_ in forward is legal
        V, v_g, (h0, c0) = enc_forward(images)
        return V, v_g, (h0.clone(), c0.clone())

    m.encoder.forward = enc_d2
    images = torch.from_numpy(feats)
    captions = torch.from_numpy(caps)
    packed = m(images, captions, lengths)                                   # baseline_attention.py:206-230
    targets = pack_padded_sequence(captions[:, 1:], lengths, batch_first=True)[0]   # train.py:101
    loss = torch.nn.CrossEntropyLoss()(packed[0], targets)                 # train.py:63,208
    m.zero_grad()
    loss.backward()                                                         # train.py:210
    out = {"captions": caps, "lengths": np.array(lengths, np.int32), "scores": packed[0].detach().numpy(),
           "batch_sizes": packed[1].numpy().astype(np.int32), "targets": targets.numpy(),
           "loss": np.array(loss.item(), np.float64)}
    grng = np.random.default_rng(7)
    for k, p in m.named_parameters():
        if k.startswith("encoder.resnet_conv"):
            continue
        g = p.grad.detach().numpy().reshape(-1) if p.grad is not None else np.zeros(p.numel(), np.float32)
        key = "g:" + k
        if g.size <= FULL_MAX:
            out[key] = g.astype(np.float32)
        else:
            idx = np.sort(grng.choice(g.size, NSAMPLE, replace=False)).astype(np.int64)
            out[key + ":idx"] = idx
            out[key] = g[idx].astype(np.float32)
        out[key + ":norm"] = np.array(np.linalg.norm(g.astype(np.float64)), np.float64)
    np.savez_compressed(os.path.join(HERE, "train_b4.npz"), **out)
    print("loss", loss.item(), "N", packed[0].shape, "params", sum(1 for k in out if k.endswith(":norm")))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Bitwise A/B of two library builds on one decode (GPU box): run once per build with AA_LIB_PATH
set, dumping the outputs; then compare the dumps.
    AA_LIB_PATH=a.so python tools/ab_bits.py dump gpurun_out/a.npz [--beam K] [--batch B]
    AA_LIB_PATH=b.so python tools/ab_bits.py dump gpurun_out/b.npz ...
    (--train bf16|fp32 --batch 128 --T 18: one training step's scores and gradients instead)
    python tools/ab_bits.py cmp gpurun_out/a.npz gpurun_out/b.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def dump_train(path, batch, T, dtype):
    """One teacher-forced forward + CE + backward (bench_train's batch): scores and every gradient."""
    import torch
    import torch.nn.functional as F
    from torch.nn.utils.rnn import pack_padded_sequence
    from bench_train import make_batch
    from adaptive_amd import Config, Encoder2Decoder
    from adaptive_amd.adaptive_attention import synthetic_features
    dev = torch.device("cuda", 0)
    caps_np, lengths = make_batch(batch, T)
    m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    m.train_bf16 = dtype == "bf16"
    m.train_aux_stream = os.environ.get("AB_ONE_STREAM") != "1"  # bitwise A/B of the two-stream calls
    feats = synthetic_features(batch, dev, seed=0)
    caps = torch.from_numpy(caps_np).to(dev)
    packed = m(feats, caps, lengths)
    loss = F.cross_entropy(packed[0], pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0])
    loss.backward()
    torch.cuda.synchronize()
    out = {"scores": packed[0].detach().cpu().numpy(), "loss": loss.detach().cpu().numpy()}
    for n, p_ in m.named_parameters():
        if p_.grad is not None:
            out["grad." + n] = p_.grad.cpu().numpy()
    np.savez(path, **out)
    print("dumped", path, len(out), "arrays")


def dump(path, beam, batch, T, fast):
    import torch
    from adaptive_amd import Config, Encoder2Decoder
    from adaptive_amd.adaptive_attention import synthetic_features
    m = Encoder2Decoder(Config()).to("cuda:0")
    m.load_synthetic(123)
    feats = synthetic_features(batch, "cuda:0", seed=0)
    if beam:
        out = m.beam_search(feats, max_len=T, beam_size=beam, fast=fast)
        names = ("ids", "alpha", "beta", "seqs", "scores")
    else:
        out = m.sampler(feats, max_len=T)
        names = ("ids", "alpha", "beta")
    torch.cuda.synchronize()
    np.savez(path, **{n: o.cpu().numpy() for n, o in zip(names, out)})
    print("dumped", path, {n: o.shape for n, o in zip(names, out)})


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    ok = True
    for n in x.files:
        same = x[n].tobytes() == y[n].tobytes()
        ok &= same
        print(n, "bit-identical" if same else f"DIFFERS (max |d| {np.abs(x[n].astype(np.float64) - y[n]).max():.3g})")
    print("ALL BIT-IDENTICAL" if ok else "DIFFERENT")
    return 0 if ok else 1


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("dump", "cmp"))
    ap.add_argument("files", nargs="+")
    ap.add_argument("--beam", type=int, default=0)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--T", type=int, default=20)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--train", choices=("bf16", "fp32"), default=None, help="dump a training step instead")
    a = ap.parse_args()
    if a.mode == "dump" and a.train:
        dump_train(a.files[0], a.batch, a.T, a.train)
    elif a.mode == "dump":
        dump(a.files[0], a.beam, a.batch, a.T, a.fast)
    else:
        sys.exit(cmp(*a.files))

#!/usr/bin/env python3
"""Training-step benchmark (BASELINE.json config 5): one train.py closure step
of Encoder2Decoder at B=128, captions of T=18 steps (+ <start>), on 1 MI355X:

    zero_grad -> forward (HIP, teacher-forced) -> CrossEntropyLoss on the packed scores
    -> backward (HIP) -> clip_grad_norm_(LSTM, 5) -> Adam step          (train.py:197-219)

The loss and the optimizer are adaptive_amd.optim's HIP CrossEntropyLoss and Adam by default (one
launch chain each, same numerics as torch's; tests/test_gpu_optim.py); --loss torch / --opt torch
run PyTorch's nn.CrossEntropyLoss / torch.optim.Adam instead.

Synthetic data: post-trunk features [B,2048,7,7] U[0,1), random captions with lengths 18 .. 9
sorted descending, random-init weights of the reference architecture.  bf16 GEMMs (fp32 accumulate,
fp32 master weights and elementwise work; BASELINE config 5) by default, --dtype fp32 for fp32 GEMMs.  Prints ONE
JSON line (steps/s; ms/step; the CPU oracle's autograd step timed on this host beside it).

    python bench_train.py [--steps 50] [--warmup 3] [--batch 128] [--T 18] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
from torch.nn.utils.rnn import pack_padded_sequence

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from adaptive_amd import Config, Encoder2Decoder, synth  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402


def make_batch(B, T, seed=0):
    rng = np.random.default_rng(seed)
    lengths = sorted(rng.integers(T // 2, T + 1, size=B).tolist(), reverse=True)
    lengths[0] = T
    caps = rng.integers(2, 10123, size=(B, T + 1)).astype(np.int64)
    caps[:, 0] = 1
    return caps, lengths


PEAK_BF16 = 2.5e15   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32 = 157.3e12


def train_flops(B, T, lengths, E=256, H=512, V=10123, C=2048, P=49):
    """Algorithmic GEMM FLOPs of one training step (forward + backward): every GEMM's
    forward product, its weight gradient and -- except the encoder's, whose input (the post-trunk
    features) needs no gradient here -- its input gradient.  Elementwise work, softmaxes, the
    attention's 49 x 49 terms and Adam are not counted."""
    R, N = B * T, int(sum(lengths))
    g = {  # name: (M, N_out, K) of the forward product
        "enc_V": (B * P, H, C), "enc_heads": (B, E + 2 * H, C), "VWv": (B * P, P, H),
        "x_terms": (R, 5 * H, 2 * E), "lstm_hh": (R, 4 * H, H), "sentinel_h": (R - B, H, H),
        "att_proj": (R, 2 * P, H), "vocab": (N, V, H)}
    fwd = sum(2 * m * n * k for m, n, k in g.values())
    bwd = sum(2 * 2 * m * n * k for m, n, k in g.values()) - 2 * B * P * H * C  # no d(features)
    ctx = 2 * R * P * H  # context sum_k alpha_k V_k (forward), counted once
    return {"total": fwd + bwd + ctx, "forward": fwd + ctx, "backward": bwd, "gemms": g}


def step(model, opt, crit, feats, caps, lengths, clip=None):
    targets = pack_padded_sequence(caps[:, 1:], lengths, batch_first=True)[0]  # train.py:102, per batch
    model.zero_grad()
    opt.zero_grad()
    packed = model(feats, caps, lengths)
    loss = crit(packed[0], targets)
    loss.backward()
    (clip or torch.nn.utils.clip_grad_norm_)(model.decoder.LSTM.parameters(), 5.0)
    opt.step()
    return loss


def cpu_baseline(caps, lengths, B, budget_s):
    from oracle.adaptive_oracle import TrainOracle  # test / baseline infrastructure only
    from bench import available_cpus  # every CPU this process may use (affinity capped by the cgroup quota)
    threads = available_cpus()["usable"]
    torch.set_num_threads(threads)
    m = TrainOracle(synth.make_weights(123))
    feats = torch.from_numpy(synth.make_features(B, seed=0))
    capst = torch.from_numpy(caps)
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 2 or (time.perf_counter() < t_end and len(times) < 5):
        t0 = time.perf_counter()
        for v in m.w.values():
            v.grad = None
        loss, _ = m.loss(feats, capst, lengths)
        loss.backward()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": 1.0 / med, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/adaptive_oracle.py TrainOracle forward + CE + autograd backward (PyTorch-CPU fp32, "
                      f"reference op order) on the same B={B} batch, no optimizer; median of {len(times)} runs "
                      f"({', '.join(f'{t:.2f}' for t in times)} s); {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--T", type=int, default=18)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="bf16",
                    help="GEMM operand type: bf16 (AA_TRAIN_BF16, BASELINE config 5) or fp32")
    ap.add_argument("--loss", choices=("hip", "torch"), default="hip",
                    help="CrossEntropyLoss: adaptive_amd.optim (HIP) or torch.nn")
    ap.add_argument("--opt", choices=("hip", "torch"), default="hip",
                    help="Adam: adaptive_amd.optim (HIP, one launch) or torch.optim (foreach)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, T = args.batch, args.T
    caps_np, lengths = make_batch(B, T)
    model = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    model.train_bf16 = args.dtype == "bf16"
    feats = synthetic_features(B, dev, seed=0)
    caps = torch.from_numpy(caps_np).to(dev)
    from adaptive_amd import optim as aa_optim
    opt = (aa_optim.Adam if args.opt == "hip" else torch.optim.Adam)(model.parameters(), lr=1e-4)
    crit = aa_optim.CrossEntropyLoss() if args.loss == "hip" else torch.nn.CrossEntropyLoss()
    clip = aa_optim.clip_grad_norm_ if args.opt == "hip" else None  # torch.nn.utils.clip_grad_norm_ otherwise
    for _ in range(args.warmup):
        step(model, opt, crit, feats, caps, lengths, clip)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        th = time.perf_counter()
        loss = step(model, opt, crit, feats, caps, lengths, clip)
        host += time.perf_counter() - th
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # host side of each step alone (the Python calls return before their kernels run): when it
    # approaches ms_per_step the step is bound by the host's launch rate, not by the GPU
    host_ms = 1e3 * host / args.steps
    out = {"metric": "training steps/s (teacher-forced fwd+bwd+Adam, B=128, T=18)", "value": args.steps / el,
           "unit": "steps/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": 1e3 * el / args.steps, "host_ms_per_step": host_ms, "higher_is_better": True,
           "dtype": args.dtype,
           "data": "synthetic: U[0,1) post-trunk features, random captions (lengths T..T/2, sorted), random-init weights",
           "config": {"workload": f"Encoder2Decoder.forward + CE + backward + clip + Adam, B={B}, T={T}",
                      "batch": B, "T": T, "packed_rows": int(sum(lengths)),
                      "gemm": "bf16 operands, fp32 accumulate (v_mfma_f32_32x32x16_bf16), fp32 master weights / Adam"
                      if args.dtype == "bf16" else "fp32 (v_mfma_f32_32x32x2f32)",
                      "loss": "adaptive_amd.optim.CrossEntropyLoss (HIP)" if args.loss == "hip" else "torch.nn.CrossEntropyLoss",
                      "optimizer": "adaptive_amd.optim.Adam + clip_grad_norm_ (HIP)" if args.opt == "hip"
                      else "torch.optim.Adam (foreach) + torch.nn.utils.clip_grad_norm_"},
           "final_loss": float(loss.item()), "cpu_baseline": None}
    fl = train_flops(B, T, lengths)
    peak = PEAK_BF16 if args.dtype == "bf16" else PEAK_FP32
    achieved = fl["total"] / (el / args.steps)
    out["roofline"] = {"kernel": "whole step (k_tgemm / k_bgemm GEMMs + elementwise + Adam)", "bound": "mfma",
                       "achieved": achieved / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s", "frac": achieved / peak,
                       "traffic": None, "flops_per_step": fl["total"],
                       "note": "algorithmic GEMM FLOPs of forward + backward (bench_train.train_flops) over the "
                               "measured step time, against the dense MFMA peak of the GEMM dtype; the dominant "
                               "kernel is k_tgemm (rocprof summary in profiles/)"}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(caps_np, lengths, B, args.cpu_budget)
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Per-workgroup phase timestamps of the fused LSTM + attention launch (tools only; round 6).

    bash tools/build_variant.sh at_ts WORK -DAA_TS_ENABLE
    AA_LIB_PATH=$PWD/abvar/at_ts.so python tools/ktrace_at.py [--flags N]

The marks of the LAST launch of a B = 512, T = 20 decode (k_lstm<512, false, true, true>): attention
role = kid 4, blocks 0..NR-1 (0 entry / rescoring start, 1 key published, 2 attention loads issued,
3 ready seen (after the drain), 4 row A done, 5 exit; slot 7 = 1 ready, 2 timed out); GEMM role = kid 0,
blocks NR.. (0 entry, 5 ring done, 1 keys + gathers, 2 tile summed, 3 cell stored, 4 tail done,
6 after the arrival / fallback; slot 7 = 1 for the row block's last arriver).  Microseconds after the
launch's earliest workgroup entry; quantiles over workgroups."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from adaptive_amd import Config, Encoder2Decoder, _lib  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402

ATT = [(0, "entry"), (1, "key published"), (2, "atten loads issued"), (3, "ready seen"), (4, "row A done"),
       (5, "exit")]
GEMM = [(0, "entry"), (5, "ring done"), (1, "keys+gathers"), (2, "tile summed"), (3, "cell stored"),
        (4, "tail done"), (6, "arrived (+fallback)")]


def q(x):
    return " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 100]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--batch", type=int, default=512)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    lib.aa_ts_setup.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(6 * 2048 * 16, dtype=torch.int64, device=dev)
    m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    m.decode_extra_flags = args.flags
    B = args.batch
    feats = synthetic_features(B, dev, seed=0)
    NR = (((B + 1) // 2) + 7) // 8 * 8
    for _ in range(3):
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.aa_ts_setup(buf.data_ptr()), "ts_setup")
        m.sampler(feats, max_len=20)
        torch.cuda.synchronize()
    ts = buf.view(6, 2048, 16).cpu().numpy().astype(np.int64)
    att = ts[4, :NR]
    gem = ts[0, NR:NR + 256]
    e = np.concatenate([att[att[:, 0] > 0, 0], gem[gem[:, 0] > 0, 0]])
    t0 = e.min()
    print(f"fused launch, B={B}: {int((att[:, 0] > 0).sum())} attention-role and {int((gem[:, 0] > 0).sum())} GEMM-role "
          f"workgroups traced; times in us after the earliest entry (min p10 p50 p90 max)")
    for name, rows, marks in (("attention role", att, ATT), ("GEMM role", gem, GEMM)):
        print(name)
        for sl, lb in marks:
            v = rows[:, sl]
            v = v[v > 0]
            if v.size:
                print(f"  {lb:22s} {q((v - t0) / 100.0)}  (n={v.size})")
    print("attention role: ready", int((att[:, 7] == 1).sum()), "timed out", int((att[:, 7] == 2).sum()))
    la = gem[gem[:, 7] == 1]
    print("GEMM role: last arrivers", len(la))
    if len(la):
        print("  last-arriver fallback span (us):", q((la[:, 6] - la[:, 4]) / 100.0))


if __name__ == "__main__":
    main()

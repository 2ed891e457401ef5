"""Per-workgroup phase timestamps of the decode-step kernels (tools only).

Build the instrumented library (s_memrealtime marks, AA_TS in the kernels) and run on the GPU box:
    make -C adaptive_amd/csrc OUT=$PWD/tools/_build/lib_ts.so CXXFLAGS="... -DAA_TS_ENABLE"
    AA_LIB_PATH=$PWD/tools/_build/lib_ts.so python tools/ktrace.py
Each kernel's marks come from its LAST launch in a B = 512, T = 20 decode (steady state).  Times
are microseconds after the kernel's earliest workgroup entry; quantiles over workgroups."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from adaptive_amd import Config, Encoder2Decoder, _lib  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402

KERNELS = {0: ("k_lstm", ["entry", "gemm done", "tile summed", "cell stored", "exit"]),
           1: ("k_atten5", ["entry", "proj barrier", "scores barrier", "softmax barrier", "exit"]),
           2: (("k_vscreen2", ["entry", "mainloop done", "exit"]) if not os.environ.get("AA_VOCAB_LISTS") else
               ("k_vscreen3", ["entry", "mainloop done", "M read", "appended"])),
           3: (("k_vrescore", ["entry", "M reduced", "candidates", "exit"]) if not os.environ.get("AA_VOCAB_LISTS") else
               ("k_vrescore3", ["entry", "listed", "exit"]))}


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    lib.aa_ts_setup.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(5 * 2048 * 16, dtype=torch.int64, device=dev)
    m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    feats = synthetic_features(512, dev, seed=0)
    for rep in range(3):
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.aa_ts_setup(buf.data_ptr()), "ts_setup")
        m.sampler(feats, max_len=20)
        torch.cuda.synchronize()
    ts = buf.view(5, 2048, 16).cpu().numpy()
    for kid, (name, marks) in KERNELS.items():
        t = ts[kid, :, :len(marks)].astype(np.int64)
        ok = t[:, 0] > 0
        if not ok.any():
            continue
        t = t[ok]
        tc = ts[kid, :, 8:8 + len(marks)].astype(np.int64)[ok]
        span_rt = (t[:, -1] - t[:, 0]).astype(np.float64)
        clk = np.median((tc[:, -1] - tc[:, 0]) / np.maximum(span_rt, 1) * 0.1)  # GHz (realtime: 100 MHz)
        t0 = t[:, 0].min()
        rel = (t - t0) * 0.01  # 100 MHz ticks -> us
        print(f"{name}: {ok.sum()} workgroups; span {rel.max():.2f} us; shader clock {clk:.2f} GHz")
        if name == "k_vscreen3":
            v = ts[kid, :, 7][ok]
            cnt, rd = v % 1000, v // 1000
            print(f"   candidates per workgroup: mean {cnt.mean():.1f}  p90 {np.quantile(cnt, 0.9):.0f}  max {cnt.max()};"
                  f"  running-max reads: mean {rd.mean():.2f} max {rd.max()}")
        for i, mk in enumerate(marks):
            q = np.quantile(rel[:, i], [0.0, 0.5, 0.9, 1.0])
            d = np.quantile(rel[:, i] - rel[:, i - 1], [0.5, 0.9]) if i else (0, 0)
            print(f"   {mk:16s} at  min {q[0]:6.2f}  med {q[1]:6.2f}  p90 {q[2]:6.2f}  max {q[3]:6.2f}   "
                  f"phase med {d[0]:5.2f} p90 {d[1]:5.2f}")


if __name__ == "__main__":
    main()

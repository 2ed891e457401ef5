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

# kid: (name, marks [(slot, label)] in time order, first workgroup index) -- the fused k_lstm<.., RS>
# launch of the last step: its GEMM workgroups are blocks NR.. (256.. at B = 512; blocks 0..255 of kid
# 0 hold step 0's plain launch), its rescoring workgroups write kid 4
KERNELS = {0: ("k_lstm (fused, GEMM role)", [(0, "entry"), (5, "ring done"), (1, "keys+gathers"), (2, "tile summed"),
                                             (3, "cell stored"), (4, "exit")], 256),
           4: ("k_lstm (fused, rescoring role)", [(0, "entry"), (1, "key published")], 0),
           1: ("k_atten5", list(enumerate(["entry", "proj barrier", "scores barrier", "softmax barrier", "exit"])), 0),
           2: ("k_vscreen8", list(enumerate(["entry", "mainloop done", "exit"])), 0),
           3: ("k_vrescore", list(enumerate(["entry", "M reduced", "candidates", "exit"])), 0)}


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    lib.aa_ts_setup.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(6 * 2048 * 16, dtype=torch.int64, device=dev)
    m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    feats = synthetic_features(512, dev, seed=0)
    for rep in range(3):
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.aa_ts_setup(buf.data_ptr()), "ts_setup")
        m.sampler(feats, max_len=20)
        torch.cuda.synchronize()
    ts = buf.view(6, 2048, 16).cpu().numpy()
    # the fused launch's two roles on one time axis: their earliest entry
    e0 = ts[0, 256:, 0][ts[0, 256:, 0] > 0]
    e4 = ts[4, :, 0][ts[4, :, 0] > 0]
    fused_t0 = min([int(x.min()) for x in (e0, e4) if x.size] or [0])
    for kid, (name, smarks, first) in KERNELS.items():
        slots = [sl for sl, _ in smarks]
        marks = [lb for _, lb in smarks]
        t = ts[kid][:, slots].astype(np.int64)
        ok = (t[:, 0] > 0) & (np.arange(2048) >= first)
        if not ok.any():
            continue
        t = t[ok]
        tc = ts[kid][:, [8 + sl for sl in slots]].astype(np.int64)[ok]
        span_rt = (t[:, -1] - t[:, 0]).astype(np.float64)
        clk = np.median((tc[:, -1] - tc[:, 0]) / np.maximum(span_rt, 1) * 0.1)  # GHz (realtime: 100 MHz)
        t0 = fused_t0 if kid in (0, 4) and fused_t0 else t[:, 0].min()
        rel = (t - t0) * 0.01  # 100 MHz ticks -> us
        print(f"{name}: {ok.sum()} workgroups; span {rel.max():.2f} us; shader clock {clk:.2f} GHz")
        for i, mk in enumerate(marks):
            q = np.quantile(rel[:, i], [0.0, 0.5, 0.9, 1.0])
            d = np.quantile(rel[:, i] - rel[:, i - 1], [0.5, 0.9]) if i else (0, 0)
            print(f"   {mk:16s} at  min {q[0]:6.2f}  med {q[1]:6.2f}  p90 {q[2]:6.2f}  max {q[3]:6.2f}   "
                  f"phase med {d[0]:5.2f} p90 {d[1]:5.2f}")


if __name__ == "__main__":
    main()

"""Sequential greedy decode with the encoder's a_g branch on a second stream (decode_aux_stream,
aa_greedy_decode_aux) against one stream, interleaved in one process (tools only; round 6).

    python tools/decode_aux_ab.py [--reps 3] [--calls 40]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from adaptive_amd import Config, Encoder2Decoder  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--calls", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    feats = synthetic_features(512, dev, seed=0)
    ref = None
    for rep in range(a.reps):
        for aux in (False, True):
            m.decode_aux_stream = aux
            for _ in range(3):
                out = m.sampler(feats, max_len=20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                out = m.sampler(feats, max_len=20)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.calls * 1e3
            same = True
            if ref is None:
                ref = out[0].clone()
            else:
                same = bool(torch.equal(ref, out[0]))
            print(f"rep {rep} aux_stream={aux}: {ms:.4f} ms per call, {512 / ms * 1e3:.0f} captions/s, ids same: {same}",
                  flush=True)


if __name__ == "__main__":
    main()

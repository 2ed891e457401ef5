"""Drive tools/kbench.hip: time individual product kernels (and variants) on a real workspace.
usage (GPU box): python tools/kbench.py [kernel ...]"""
import ctypes
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from adaptive_amd import Config, Encoder2Decoder, _lib  # noqa: E402
from adaptive_amd.adaptive_attention import synthetic_features  # noqa: E402

SO = os.path.join(ROOT, "tools", "_build", "libkbench.so")


def main():
    names = sys.argv[1:] or ["lstm", "atten", "vscreen", "vrescore"]
    if not os.path.exists(SO):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                               "-fPIC", "-shared", "-I" + os.path.join(ROOT, "include"),
                               os.path.join(ROOT, "tools", "kbench.hip"), "-o", SO])
    dev = torch.device("cuda", 0)
    model = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
    B, T = 512, 20
    feats = synthetic_features(B, dev, seed=0)
    model.sampler(feats, max_len=T)
    torch.cuda.synchronize()
    libs = {}
    for key, path in (("", SO), ("old:", os.environ.get("KB_SO_OLD", ""))):  # "old:<name>" -> a second build
        if path:
            lb = ctypes.CDLL(path)
            lb.kb_time.restype = ctypes.c_int
            lb.kb_time.argtypes = [ctypes.POINTER(_lib.Model), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
            libs[key] = lb
    m = model._model_struct()
    rounds = int(os.environ.get("KB_ROUNDS", "5"))
    res = {n: [] for n in names}
    for _ in range(rounds):  # interleaved rounds: variants see the same clocks / cache states
        for n in names:
            out = ctypes.c_float()
            reps = 20 if n.startswith("enc") else 200
            lib, kn = (libs["old:"], n[4:]) if n.startswith("old:") else (libs[""], n)
            rc = lib.kb_time(m, feats.data_ptr(), model._ws.data_ptr(), B, T, kn.encode(), reps, ctypes.byref(out))
            if rc:
                print(f"{n}: rc={rc}", flush=True)
            res[n].append(out.value)
    for n in names:
        v = sorted(res[n])
        print(f"{n:24s} median {v[len(v) // 2]:8.2f} us  min {v[0]:8.2f}  max {v[-1]:8.2f}", flush=True)


if __name__ == "__main__":
    main()

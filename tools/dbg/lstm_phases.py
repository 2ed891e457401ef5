import ctypes, os, sys
import numpy as np
sys.argv = ["kbench", "ld_m8"]
os.environ["KB_ROUNDS"] = "1"
sys.path.insert(0, "tools")
import kbench
kbench.main()
lib = ctypes.CDLL(kbench.SO)
buf = (ctypes.c_ulonglong * (256 * 8 * 8))()
print("rc", lib.kb_dbg(buf))
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8, 8).astype(np.int64)
t0 = a[:, :, 0].min()
rel = a - a[:, :, :1]
print("kernel span (cycles)", a[:, :, 6].max() - t0)
print("WG start spread", np.percentile(a[:, 0, 0] - t0, [0, 50, 100]))
for i, name in enumerate(["start", "gemm issued", "sync1 (waves4-7 stored)", "sync2 (add+Wsl)", "sync3 (4-way sum)", "sync4 (cell+stores)", "end (proj)"]):
    print(f"{name:28s} median {np.median(rel[:, :, i]):8.0f}  p90 {np.percentile(rel[:, :, i], 90):8.0f}")

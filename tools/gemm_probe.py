"""Library bf16 GEMM times for the training step's large shapes (tools only): torch.mm on bf16
operands (hipBLASLt underneath), fp32 output where torch offers it, as a yardstick for the
hand-written k_bgemm / k_tgemm<true> times in the training kernel trace.

    python tools/gemm_probe.py
"""
import torch

SHAPES = {  # name: (M, N, K) of C[M, N] = A[M, K] B[N, K]^T
    "vocab fwd (scores = U W_m^T)": (1741, 10123, 512),
    "dU = dS W_m": (1741, 512, 10123),
    "dW_m = dS^T U": (10123, 512, 1741),
    "dW_a = dV^T A": (512, 2048, 6272),
    "V = A W_a^T": (6272, 512, 2048),
    "LSTM ih fwd": (1741, 2048, 1024),
    "dW_ih = dG^T X": (2048, 1024, 1741),
    "dX = dG W_ih": (1741, 1024, 2048),
    "dW_hh = dG^T H": (2048, 512, 1741),
}


def bench(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    for name, (M, N, K) in SHAPES.items():
        a = torch.randn(M, K, device=dev).bfloat16()
        b = torch.randn(N, K, device=dev).bfloat16()
        t16 = bench(lambda: torch.mm(a, b.t()))
        try:
            t32 = bench(lambda: torch.mm(a, b.t(), out_dtype=torch.float32))
        except Exception as ex:  # noqa: BLE001
            t32 = float("nan")
            err = type(ex).__name__
        else:
            err = ""
        fl = 2.0 * M * N * K
        print(f"{name:32s} M={M:6d} N={N:6d} K={K:6d}  bf16-out {t16:8.1f} us ({fl / t16 / 1e6:7.1f} TF/s)"
              f"  fp32-out {t32:8.1f} us ({fl / t32 / 1e6:7.1f} TF/s) {err}")


if __name__ == "__main__":
    main()

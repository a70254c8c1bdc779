"""Roofline lines for the wide-MLP kernels (csrc/kernels/wlin.hip) at SAC1024Policy sizes
([1024, 1024] hidden, reference scripts/ingredients/policy.py SAC1024 policy) and at the
MultiBC [256, 256, 128] sizes: per-layer forward (GEMM + bias + act), dW / db and dX launches,
timed with HIP events over many replays, against rocBLAS/hipBLASLt (torch bf16 matmul) of the
same GEMM and the dense bf16 MFMA peak (2.5 PFLOP/s) / HBM (8 TB/s).

    python tools/wlin_roofline.py > profiles/r4_wlin_roofline.md
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch as th

PEAK_TF = 2500.0  # dense bf16 TFLOP/s
HBM_TBS = 8.0


def timeit(fn, n=200, warm=20):
    for _ in range(warm):
        fn()
    th.cuda.synchronize()
    e0, e1 = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    th.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


def main():
    from imitation_amd.ops import native

    C = native()
    dev = th.device("cuda")
    th.manual_seed(0)
    print("| layer (M x K -> N) | op | us | TFLOP/s | % bf16 peak | GB/s (min bytes) | torch bf16 matmul us |")
    print("|---|---|---|---|---|---|---|")
    shapes = []
    for M in (256, 1024, 4096):  # SAC batch 256; larger rows: replay / ensemble batches
        shapes += [(M, 17, 1024, "SAC1024 layer 0"), (M, 1024, 1024, "SAC1024 layer 1"), (M, 1024, 6, "SAC1024 head")]
    shapes += [(1024, 48, 256, "MultiBC layer 0"), (1024, 256, 256, "MultiBC layer 1"), (1024, 256, 128, "MultiBC layer 2")]
    for M, K, N, name in shapes:
        x = th.randn(M, K, device=dev)
        w = th.randn(N, K, device=dev) * K ** -0.5
        b = th.randn(N, device=dev)
        h = C.wlin_forward(x, w, b, 1)
        dz = th.randn(M, N, device=dev)
        flops = 2.0 * M * K * N
        xb, wb = x.bfloat16(), w.bfloat16()
        t_ref = timeit(lambda: th.matmul(xb, wb.t()))
        for op, fn, byt in (
            ("fwd", lambda: C.wlin_forward(x, w, b, 1), 4 * (M * K + N * K + M * N)),
            ("dW+db", lambda: C.wlin_backward_w(dz, x, True), 4 * (M * N + M * K + N * K)),
            ("dX", lambda: C.wlin_backward_x(dz, w, x, 1, None), 4 * (M * N + N * K + 2 * M * K)),
        ):
            us = timeit(fn)
            tf = flops / us * 1e-6
            print(f"| {name} ({M} x {K} -> {N}) | {op} | {us:.2f} | {tf:.1f} | {100 * tf / PEAK_TF:.2f} | "
                  f"{byt / us * 1e-3:.0f} | {t_ref:.2f} |", flush=True)
        del h


if __name__ == "__main__":
    main()

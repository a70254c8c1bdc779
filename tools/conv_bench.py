"""NatureCNN conv trunk fwd+bwd: HIP NHWC kernels vs MIOpen (torch fp32 NCHW, torch bf16 channels_last).

Prints ms per fwd+bwd for batch sizes 32 / 256 / 1024 (Pong frames 84x84x4).
"""
import sys
import time

import torch as th
import torch.nn.functional as F

import os  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imitation_amd.ops import conv as conv_ops  # noqa: E402

LAYERS = [((32, 4, 8, 8), 4), ((64, 32, 4, 4), 2), ((64, 64, 3, 3), 1)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    th.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


def main():
    ws = [(th.randn(s, device="cuda") * 0.05).requires_grad_(True) for s, _ in LAYERS]
    bs = [th.zeros(s[0], device="cuda", requires_grad=True) for s, _ in LAYERS]
    ss = [st for _, st in LAYERS]
    for B in (32, 256, 1024):
        x = th.rand(B, 84, 84, 4, device="cuda")
        gy = th.randn(B, 7, 7, 64, device="cuda")

        def hip():
            y = conv_ops.conv_stack(x, ws, bs, ss)
            th.autograd.grad((y * gy).sum(), ws + bs)

        def ref32():
            y = conv_ops.conv_stack_reference(x, ws, bs, ss)
            th.autograd.grad((y * gy).sum(), ws + bs)

        xb = x.permute(0, 3, 1, 2).contiguous(memory_format=th.channels_last).bfloat16()

        def ref16():
            h = xb
            for w, b, s in zip(ws, bs, ss):
                h = F.relu(F.conv2d(h, w.bfloat16(), b.bfloat16(), stride=s))
            th.autograd.grad((h.float().permute(0, 2, 3, 1) * gy).sum(), ws + bs)

        t_h, t_32, t_16 = timeit(hip), timeit(ref32), timeit(ref16)
        print(f"B={B}: hip {t_h:.3f} ms | miopen fp32 {t_32:.3f} ms | miopen bf16 channels_last {t_16:.3f} ms", flush=True)


if __name__ == "__main__":
    main()

"""Reward CNN (CnnRewardNet defaults: 3x3 stride-1 'same' conv + ReLU, 32 -> 32 channels, on
Pong frames 84x84x4) fwd+bwd: HIP NHWC padded kernels vs MIOpen (torch fp32 NCHW, torch bf16
channels_last). Prints ms per fwd+bwd (weight gradients) for a few batch sizes."""
import os
import sys
import time

import torch as th
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imitation_amd.ops import conv as conv_ops  # noqa: E402


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    th.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


def main():
    th.manual_seed(0)
    ws = [(th.randn(32, 4, 3, 3, device="cuda") * 0.2).requires_grad_(), (th.randn(32, 32, 3, 3, device="cuda") * 0.1).requires_grad_()]
    bs = [th.zeros(32, device="cuda", requires_grad=True) for _ in range(2)]
    for B in (32, 128, 512):
        x = th.rand(B, 84, 84, 4, device="cuda")
        gy = th.randn(B, 84, 84, 32, device="cuda")
        gyb = gy.bfloat16()

        def hip():
            y = conv_ops.conv_stack(x, ws, bs, [1, 1], 1.0, [1, 1], out_dtype=th.bfloat16)
            th.autograd.grad((y * gyb).sum(), ws + bs)

        def ref32():
            y = conv_ops.conv_stack_reference(x, ws, bs, [1, 1], 1.0, [1, 1])
            th.autograd.grad((y * gy).sum(), ws + bs)

        xb = x.permute(0, 3, 1, 2).contiguous(memory_format=th.channels_last).bfloat16()

        def ref16():
            h = xb
            for w, b in zip(ws, bs):
                h = F.relu(F.conv2d(h, w.bfloat16(), b.bfloat16(), padding=1))
            th.autograd.grad((h.permute(0, 2, 3, 1) * gyb).sum(), ws + bs)

        t_h, t_32, t_16 = timeit(hip), timeit(ref32), timeit(ref16)
        print(f"B={B}: hip {t_h:.3f} ms | miopen fp32 {t_32:.3f} ms | miopen bf16 channels_last {t_16:.3f} ms", flush=True)


if __name__ == "__main__":
    main()

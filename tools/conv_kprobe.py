"""Our conv kernels only (for rocprof): NatureCNN trunk fwd+bwd at B=1024 and the reward CNN
(3x3 same, 4->32->32) fwd+bwd at B=512, 10 iterations each."""
import os
import sys

import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imitation_amd.ops import conv as conv_ops  # noqa: E402


def main():
    th.manual_seed(0)
    nat = [((32, 4, 8, 8), 4), ((64, 32, 4, 4), 2), ((64, 64, 3, 3), 1)]
    for layers, B, HW, pads in ((nat, 1024, 84, [0, 0, 0]), ([((32, 4, 3, 3), 1), ((32, 32, 3, 3), 1)], 512, 84, [1, 1])):
        ws = [(th.randn(s, device="cuda") * 0.05).requires_grad_() for s, _ in layers]
        bs = [th.zeros(s[0], device="cuda", requires_grad=True) for s, _ in layers]
        ss = [st for _, st in layers]
        x = th.rand(B, HW, HW, 4, device="cuda")
        y = conv_ops.conv_stack(x, ws, bs, ss, 1.0, pads, out_dtype=th.bfloat16)
        gy = th.randn_like(y)
        for _ in range(10):
            y = conv_ops.conv_stack(x, ws, bs, ss, 1.0, pads, out_dtype=th.bfloat16)
            th.autograd.grad((y * gy).sum(), ws + bs)
        th.cuda.synchronize()
        print("done", B, flush=True)


if __name__ == "__main__":
    main()

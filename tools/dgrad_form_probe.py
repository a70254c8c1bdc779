"""Time the BC-size conv backward pieces per form: conv_dgrad plain / prefetch / split-tap, the
weight-gradient partials, and the paired launch (conv_backward_pair), for NatureCNN conv2 / conv3 at
batch 32. Each case is 50 launches captured in one HIP graph, replayed 20 times; us per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402


def timed(fn, reps=50, iters=20):
    s = th.cuda.Stream()
    s.wait_stream(th.cuda.current_stream())
    with th.cuda.stream(s):
        for _ in range(3):
            fn()
    th.cuda.current_stream().wait_stream(s)
    g = th.cuda.CUDAGraph()
    with th.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    th.cuda.synchronize()
    e0, e1 = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    th.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / (reps * iters)


def main():
    from imitation_amd import ops

    Cn = ops.native()
    for name, (B, C, N, KH, S, H) in (("conv2", (32, 32, 64, 4, 2, 20)), ("conv3", (32, 64, 64, 3, 1, 9))):
        g = th.Generator().manual_seed(1)
        OH = (H - KH) // S + 1
        x = th.relu(th.randn(B, H, H, C, generator=g)).to(th.bfloat16).cuda()
        y = th.randn(B, OH, OH, N, generator=g).to(th.bfloat16).cuda()
        dy = th.randn(B, OH, OH, N, generator=g).to(th.bfloat16).cuda()
        w = (th.randn(N, C, KH, KH, generator=g) * 0.05).cuda()
        _, wts = Cn.conv_pack_weights([w], [True])
        row = {}
        for fname, form in (("plain", 0), ("pf", 1), ("split", 2)):
            row[fname] = timed(lambda: Cn.conv_dgrad(dy, y, wts[0], x, S, True, True, 0, form))
        row["wgrad"] = timed(lambda: Cn.conv_wgrad_partials(x, dy, y, KH, KH, S, 1.0, True, 0))
        row["pair"] = timed(lambda: Cn.conv_backward_pair(x, dy, y, wts[0], S, True))
        print(name, " ".join(f"{k}={v:.2f}us" for k, v in row.items()), flush=True)


if __name__ == "__main__":
    main()

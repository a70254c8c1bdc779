"""bc_head_train alone: us per launch with the NatureCNN parameter bucket (1.7M floats) and with a
tiny bucket (isolates the ||theta||^2 blocks), B=32, NH=512, A=6."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch as th  # noqa: E402


def main():
    from imitation_amd import ops

    C = ops.native()
    dev = "cuda"
    h = th.rand(32, 512, device=dev)
    W = th.randn(6, 512, device=dev) * 0.01
    b = th.zeros(6, device=dev)
    acts = th.randint(0, 6, (32,), device=dev)
    for n in (1_700_000, 4096):
        params = th.randn(n, device=dev)
        dW, db = th.zeros_like(W), th.zeros_like(b)
        m = th.zeros(8, device=dev)
        ws = th.zeros(int(C.bc_head_workspace(n)), device=dev)
        for _ in range(20):
            C.bc_head_train(h, W, b, acts, params, dW, db, m, ws, 1e-3, 0.0)
        th.cuda.synchronize()
        e0, e1 = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            C.bc_head_train(h, W, b, acts, params, dW, db, m, ws, 1e-3, 0.0)
        e1.record()
        th.cuda.synchronize()
        print(f"n_params={n}: {1e3 * e0.elapsed_time(e1) / 200:.2f} us per launch (stream-serialised)", flush=True)
        prof = th.zeros(8, dtype=th.int64, device=dev)
        C.bc_head_train(h, W, b, acts, params, dW, db, m, ws, 1e-3, 0.0, prof)
        th.cuda.synchronize()
        p = prof.cpu().tolist()
        names = ["h loads + W staged", "logit partials", "reduce", "softmax", "dW/dh", "metrics + hand-off"]
        print("  block 0 cycles: " + ", ".join(f"{nm} {p[i + 1] - p[i]}" for i, nm in enumerate(names) if p[i + 1]), flush=True)


if __name__ == "__main__":
    main()

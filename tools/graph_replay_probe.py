"""How much does a HIP-graph replay boundary cost on this ROCm? (DAgger BC epochs replay one
16-step graph back to back; the kernel trace shows ~340 us idle between replays.)

Captures a graph of `--nodes` small kernels (an elementwise add chain on a 32K-float tensor),
replays it `--reps` times back to back (one instance) and alternating between two captured
instances, and reports wall ms per replay and per node against eager launches of the same work.
Also times the host side of one replay() call."""
import argparse
import json
import time

import torch as th


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nodes", type=int, default=300)
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--numel", type=int, default=32768)
    args = p.parse_args()
    dev = th.device("cuda", 0)
    x = th.zeros(args.numel, device=dev)

    def work():
        for _ in range(args.nodes):
            x.add_(1.0)

    s = th.cuda.Stream()
    s.wait_stream(th.cuda.current_stream())
    with th.cuda.stream(s):
        work()  # warm-up
    th.cuda.current_stream().wait_stream(s)
    th.cuda.synchronize()
    graphs = []
    for _ in range(2):
        g = th.cuda.CUDAGraph()
        with th.cuda.graph(g):
            work()
        graphs.append(g)
    th.cuda.synchronize()
    out = dict(nodes=args.nodes, reps=args.reps)

    def timed(fn):
        th.cuda.synchronize()
        t0 = time.perf_counter()
        host = fn()
        th.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / args.reps, host

    def eager():
        for _ in range(args.reps):
            work()

    def same():
        t = 0.0
        for _ in range(args.reps):
            a = time.perf_counter()
            graphs[0].replay()
            t += time.perf_counter() - a
        return t * 1e3 / args.reps

    def alternate():
        t = 0.0
        for i in range(args.reps):
            a = time.perf_counter()
            graphs[i % 2].replay()
            t += time.perf_counter() - a
        return t * 1e3 / args.reps

    for name, fn in (("eager", eager), ("graph_same", same), ("graph_alternate", alternate), ("graph_same_2", same)):
        ms, host = timed(fn)
        out[name] = dict(ms_per_rep=round(ms, 4), us_per_node=round(1e3 * ms / args.nodes, 3),
                         host_ms_per_replay=None if host is None else round(host, 4))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

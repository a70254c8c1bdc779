"""Round 6: the bench trainer's timed rounds alternate fast / slow between successive trainer
instances in ONE process (2.74 / 3.43 / 3.40 / 2.74 / 3.39 / 2.72 ms per round,
``tools/expert_inproc_probe.py``). This runs two instances back to back and prints the device
addresses of the engine's buffers (placement is what differs between instances); under
``rocprofv3 --kernel-trace`` the two instances' kernels are split at the largest idle gap by
``--split <kernel_trace.csv>`` and compared per kernel.

    python tools/alt_slow_probe.py
    python tools/alt_slow_probe.py --split run_kernel_trace.csv
"""

import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def trainers(n=3):
    import torch as th

    from imitation_amd import models

    for i in range(n):
        b = models.build("gail_halfcheetah", device="cuda", env_id="HalfCheetah-v4")
        tr = b.trainer
        spr = tr.gen_train_timesteps
        tr.train(3 * spr)
        th.cuda.synchronize()
        t0 = time.perf_counter()
        tr.train(20 * spr)
        th.cuda.synchronize()
        ms = 1000 * (time.perf_counter() - t0) / 20
        bufs = {k: v for k, v in vars(tr).items() if isinstance(v, th.Tensor) and v.is_cuda}
        bufs.update({f"buf.{k}": v for k, v in getattr(tr, "buf", {}).items() if isinstance(v, th.Tensor)})
        lines = sorted((v.data_ptr(), k, v.numel() * v.element_size()) for k, v in bufs.items())
        print(f"instance {i}: {ms:.3f} ms/round", flush=True)
        for ptr, k, nb in lines:
            print(f"   {k:32s} 0x{ptr:x} (mod 2M: 0x{ptr % (2 << 20):06x}, mod 64K: 0x{ptr % 65536:05x}) {nb} B", flush=True)
        del b, tr
        time.sleep(0.5)  # an idle gap in the kernel trace between instances


def split(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    gaps = sorted(((rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)), reverse=True)
    cuts = sorted(i for _, i in gaps[:2])  # the two sleeps between three instances
    parts = [rows[: cuts[0] + 1], rows[cuts[0] + 1 : cuts[1] + 1], rows[cuts[1] + 1 :]]
    stats = []
    for p in parts:
        d = {}
        for s, e, k in p:
            d.setdefault(k[:70], []).append(e - s)
        stats.append(d)
    keys = sorted(set().union(*stats), key=lambda k: -sum(stats[0].get(k, [0])))
    print("| kernel | " + " | ".join(f"inst {i} calls / us per call" for i in range(len(stats))) + " |")
    print("|---|" + "---|" * len(stats))
    for k in keys[:20]:
        cells = []
        for d in stats:
            v = d.get(k, [])
            cells.append(f"{len(v)} / {sum(v) / max(1, len(v)) / 1000:.1f}")
        print(f"| `{k}` | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--split":
        split(sys.argv[2])
    else:
        trainers()

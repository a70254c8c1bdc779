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


def split(path, api_path=None):
    """Per instance (split at the PPO kernels: 23 per instance), over its 20 timed rounds: GPU busy
    time vs span (idle = host not keeping the queue full), and per-kernel mean durations; with
    ``api_path`` (``--hip-trace`` CSV) the slowest HIP API calls of each instance's window."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ppo = [i for i, r in enumerate(rows) if "ppo_rc_kernel" in r[2]]
    n_inst = len(ppo) // 23
    print(f"{len(ppo)} PPO kernels -> {n_inst} instances")
    windows = []
    for k in range(n_inst):
        first_timed = rows[ppo[23 * k + 3]][0]  # rounds 3..22 of the instance are the timed ones
        last = rows[ppo[23 * k + 22]][1]
        sel = [r for r in rows if first_timed <= r[0] and r[1] <= last]
        busy, cur_end = 0, 0
        for s_, e_, _ in sel:  # union of kernel intervals
            if e_ <= cur_end:
                continue
            busy += e_ - max(s_, cur_end)
            cur_end = e_
        span = last - first_timed
        windows.append((first_timed, last))
        print(f"instance {k}: span {span / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms, idle {100 * (1 - busy / span):.1f} %, "
              f"{len(sel)} kernels")
        d = {}
        for s_, e_, name in sel:
            d.setdefault(name[:60], []).append(e_ - s_)
        top = sorted(d.items(), key=lambda kv: -sum(kv[1]))[:6]
        print("   " + "; ".join(f"{n}: {len(v)} x {sum(v) / len(v) / 1000:.1f} us" for n, v in top))
    if api_path:
        calls = []
        with open(api_path) as f:
            for r in csv.DictReader(f):
                calls.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", r.get("Kernel_Name", ""))))
        for k, (a_, b_) in enumerate(windows):
            sel = [c for c in calls if a_ <= c[0] <= b_]
            d = {}
            for s_, e_, name in sel:
                d.setdefault(name, []).append(e_ - s_)
            top = sorted(d.items(), key=lambda kv: -sum(kv[1]))[:8]
            print(f"instance {k} HIP API: " + "; ".join(f"{n}: {len(v)} x {sum(v) / len(v) / 1000:.1f} us" for n, v in top))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--split":
        split(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        trainers()

"""Host/GPU interplay of the DAgger collector from a rocprofv3 `--kernel-trace --hip-trace`
database: for the idle gaps (> `min_gap` us) on the collector's queue, the HIP API calls the host
made during the gap (name, start offset, duration). Prints a small text report (the database
itself is too large to keep). Usage: dagger_api_gaps.py run.db [min_gap_us]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
    c = sqlite3.connect(db)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    kname = "name" if "name" in kcols else "kernel_name"
    ks = sorted(c.execute(f"select {kname}, start, end, queue_id from kernels").fetchall(), key=lambda r: r[1])
    rcols = [r[1] for r in c.execute("pragma table_info(regions)")]
    print("regions columns:", rcols)
    tcol = "tid" if "tid" in rcols else "0"
    rs = sorted(c.execute(f"select name, start, end, {tcol} from regions").fetchall(), key=lambda r: r[1])
    names = collections.Counter(r[0] for r in rs)
    print("API calls:", len(rs), "top:", names.most_common(12))
    env_q = collections.Counter(r[3] for r in ks if "dagger_env" in r[0]).most_common(1)[0][0]
    envs = [r for r in ks if r[3] == env_q and "dagger_env" in r[0]]
    t_from = envs[int(len(envs) * 0.6)][1]  # the timed round(s): skip start-up and warm-up
    seq = [r for r in ks if r[3] == env_q and r[1] >= t_from]
    noise = {"hipGetDevice", "hipSetDevice", "hipGetLastError", "hipStreamGetCaptureInfo", "hipStreamIsCapturing",
             "__hipPushCallConfiguration", "__hipPopCallConfiguration", "hipDevicePrimaryCtxGetState"}
    late = collections.Counter()
    for r in rs:
        if r[1] >= t_from:
            late[r[0]] += r[2] - r[1]
    print("API time after the start of the timed collection (ms):",
          [(n, round(v / 1e6, 2)) for n, v in late.most_common(12)])
    gaps = []
    for a, b in zip(seq, seq[1:]):
        g = (b[1] - a[2]) / 1e3
        if g > min_gap:
            gaps.append((a, b, g))
    print(f"gaps > {min_gap} us on the collector queue: {len(gaps)}, total {sum(g for _, _, g in gaps) / 1e3:.1f} ms")
    import bisect

    starts = [r[1] for r in rs]
    for a, b, g in sorted(gaps, key=lambda x: -x[2])[:12]:
        print(f"\n-- gap {g:.0f} us after {a[0][:50]} -> {b[0][:50]}")
        i = bisect.bisect_left(starts, a[2] - 50_000)
        while i < len(rs) and rs[i][1] < b[1]:
            n, s, e, tid = rs[i]
            if n not in noise and (e - s > 5_000 or rs[i][1] > a[2]):
                print(f"   {(s - a[2]) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  tid {tid}  {n}")
            i += 1


if __name__ == "__main__":
    main()

"""Kernel timeline of a rocprofv3 rocpd sqlite database: every dispatch between the Nth and
(N+1)th occurrence of a marker kernel (default: the rollout chain), with start offset, duration
and the idle gap before it (us). Usage: prof_timeline.py run.db [marker-substring] [N]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "rollout_chain_kernel"
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    qcol = "queue_id" if "queue_id" in cols else "0"
    rows = sorted(c.execute(f"select {name_col}, start, end, {qcol} from kernels").fetchall(), key=lambda r: r[1])
    qids = {q: i for i, q in enumerate(sorted({r[3] for r in rows}))}
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) <= nth:
        print("not enough marker dispatches", len(idx))
        return
    a, b = idx[nth], idx[nth + 1]
    t0 = rows[a][1]
    prev_end = rows[a - 1][2] if a > 0 else t0
    print(f"round between dispatch {a} and {b}: {(rows[b][1] - t0) / 1e3:.1f} us")
    print("| start us | dur us | gap us | queue | kernel |\n|---|---|---|---|---|")
    busy_end = prev_end
    for n, s, e, q in rows[a:b + 1]:
        gap = (s - busy_end) / 1e3
        short = n if len(n) < 80 else n[:77] + "..."
        print(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {gap:.1f} | q{qids[q]} | `{short}` |")
        busy_end = max(busy_end, e)


if __name__ == "__main__":
    main()

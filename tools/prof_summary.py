"""Summarise a rocprofv3 rocpd sqlite database into a kernel-time table (markdown)."""
import sqlite3, sys
db = sys.argv[1]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = 'name' if 'name' in cols else ('kernel_name' if 'kernel_name' in cols else None)
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = {}
t0 = min(r[1] for r in rows); t1 = max(r[2] for r in rows)
for n, s, e in rows:
    d = agg.setdefault(n, [0, 0.0])
    d[0] += 1; d[1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"kernels: {len(rows)} dispatches, busy {tot/1e3:.2f} ms over a {((t1-t0)/1e6):.2f} ms window\n")
print("| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|")
for n, (k, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    short = n if len(n) < 90 else n[:87] + '...'
    print(f"| `{short}` | {k} | {us:.1f} | {us/k:.2f} | {100*us/tot:.1f} |")

# one round of the headline: the dispatches between two consecutive PPO-kernel starts (the
# middle pair of the trace), with their start / duration / gap to the previous kernel's end
if len(sys.argv) > 3 and sys.argv[3] == "round":
    rows.sort(key=lambda r: r[1])
    ppo = [i for i, r in enumerate(rows) if "ppo_rc_kernel" in r[0]]
    if len(ppo) >= 3:
        a, b = ppo[len(ppo) // 2 - 1], ppo[len(ppo) // 2]
        base = rows[a][1]
        print(f"\n## One headline round\n\nround between dispatch {a} and {b}: {(rows[b][1] - base) / 1e3:.1f} us\n")
        print("| start us | dur us | gap us | kernel |\n|---|---|---|---|")
        prev_end = None
        for n, s, e in rows[a:b + 1]:
            gap = 0.0 if prev_end is None else (s - prev_end) / 1e3
            short = n if len(n) < 80 else n[:77] + '...'
            print(f"| {(s - base) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {gap:.1f} | `{short}` |")
            prev_end = e if prev_end is None else max(prev_end, e)

"""Summarise a rocprofv3 `--kernel-trace --marker-trace` database of a run with
IMITATION_AMD_ROCTX=1: host time per ROCTX range name (count, total, mean), then one steady-state
round (the Nth occurrence of `--round-range`) as a host-range + device-kernel timeline. Prints a
small markdown report: the database itself is too large to keep.

Usage: roctx_summary.py run.db [--round-range NAME] [--nth N]"""
import argparse
import collections
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--round-range", default="ppo/update")
    p.add_argument("--nth", type=int, default=6)
    args = p.parse_args()
    c = sqlite3.connect(args.db)
    rcols = [r[1] for r in c.execute("pragma table_info(regions)")]
    cat = "category" if "category" in rcols else "''"
    # a ROCTX range's region name is the API (roctxThreadRangeA...), its text is extdata's message
    msg = "coalesce(json_extract(extdata, '$.message'), name)" if "extdata" in rcols else "name"
    regions = c.execute(f"select {msg}, start, end, {cat} from regions").fetchall()
    markers = [r for r in regions if not str(r[0]).startswith("hip") and not str(r[0]).startswith("__hip")]
    print(f"{len(markers)} ROCTX ranges, categories {collections.Counter(r[3] for r in markers).most_common(4)}\n")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e, _ in markers:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
    print("| range | count | total ms | mean us |\n|---|---|---|---|")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"| `{n}` | {k} | {t / 1e3:.2f} | {t / k:.1f} |")
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    kname = "name" if "name" in kcols else "kernel_name"
    ks = sorted(c.execute(f"select {kname}, start, end from kernels").fetchall(), key=lambda r: r[1])
    rounds = sorted([r for r in markers if r[0] == args.round_range], key=lambda r: r[1])
    if len(rounds) <= args.nth + 1:
        print(f"\n(fewer than {args.nth + 2} `{args.round_range}` ranges)")
        return
    t0, t1 = rounds[args.nth][1], rounds[args.nth + 1][1]
    print(f"\n## One round: `{args.round_range}` #{args.nth} to #{args.nth + 1} ({(t1 - t0) / 1e3:.1f} us of host time)\n")
    print("| host t us | host dur us | range |\n|---|---|---|")
    for n, s, e, _ in sorted(markers, key=lambda r: r[1]):
        if t0 <= s < t1:
            print(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | `{n}` |")
    print("\n| device t us | dur us | kernel |\n|---|---|---|")
    shown = 0
    for n, s, e in ks:
        if t0 <= s < t1 and (e - s) > 5_000 and shown < 60:
            short = n if len(n) < 70 else n[:67] + "..."
            print(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | `{short}` |")
            shown += 1


if __name__ == "__main__":
    main()

"""Per-kernel instruction census of a hipcc ``-S`` dump (spills, MFMA, LDS, waits).

usage: python tools/isa_stats.py file.s [name-substring]
"""
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l) and pat in l]
    keys = ["scratch_", "v_writelane", "v_readlane", "v_mfma", "ds_read", "ds_write", "s_waitcnt", "global_load", "s_barrier",
            "v_accvgpr"]
    for st in starts:
        en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
        body = lines[st:en]
        cnt = {k: sum(1 for l in body if k in l) for k in keys}
        print(lines[st].split(":")[0][-60:], "lines", len(body), " ".join(f"{k}={v}" for k, v in cnt.items()))


if __name__ == "__main__":
    main()

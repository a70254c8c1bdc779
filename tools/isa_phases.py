"""Static instruction mix of the rollout chain's step, per phase.

The phase-clock instance of ``rollout_chain_kernel`` (``PROF = true``, rollout.hip) brackets each
step's phases with ``s_memtime`` stamps; this splits that kernel's assembly at the stamps (program
order, the step body is straight-line code between them apart from the reset branch) and counts
instruction classes per phase. Run on the host:

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/kernels -Icsrc/runtime \
        --cuda-device-only -S -o /tmp/rollout.s csrc/kernels/rollout.hip
    python tools/isa_phases.py /tmp/rollout.s
"""

import re
import sys
from collections import Counter

PHASES = ("actor + sampling", "env physics (5 substeps)", "observation", "step tail (stores, reset test)")


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_rcp", "v_sin", "v_cos", "v_log", "v_sqrt", "v_rsq")):
        return "valu_trans"
    if "_dpp" in op or op.startswith(("v_permlane", "v_readlane", "v_readfirstlane", "v_writelane")):
        return "cross_lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_barrier", "s_cbranch", "s_branch")):
        return "branch/barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, kernel_pat=r"rollout_chain_kernelILb1ELi2ELi2ELi3ELi32ELi5ELb1E"):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{kernel_pat}\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = [l.strip() for l in lines[start:end]]
    stamps = [i for i, l in enumerate(body) if l.startswith("s_memtime")]
    if len(stamps) < 5:
        raise SystemExit(f"expected >= 5 s_memtime stamps, found {len(stamps)}")
    s0 = stamps[:5]  # t0 t1 t2 t3 t4 of the step body, program order
    print(f"kernel {kernel_pat}: {end - start} lines, {len(stamps)} stamps")
    print(f"| phase | instructions | " + " | ".join(("valu", "valu_trans", "cross_lane", "lds", "vmem", "salu", "waitcnt", "branch/barrier")) + " |")
    print("|---|---|" + "---|" * 8)
    for k, name in enumerate(PHASES):
        seg = body[s0[k] + 1:s0[k + 1]]
        ops = [l.split()[0] for l in seg if l and not l.startswith((";", ".")) and not l.endswith(":")]
        c = Counter(klass(o) for o in ops)
        print(f"| {name} | {len(ops)} | " + " | ".join(str(c.get(x, 0)) for x in
                                                      ("valu", "valu_trans", "cross_lane", "lds", "vmem", "salu", "waitcnt", "branch/barrier")) + " |")


if __name__ == "__main__":
    main(*sys.argv[1:])

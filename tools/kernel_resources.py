"""Register / scratch / LDS budget of every kernel instance of the given HIP sources.

Compiles each source for gfx950 with ``-Rpass-analysis=kernel-resource-usage`` (device only,
no object kept) and prints one markdown table row per kernel instance: VGPRs, AGPRs, SGPRs,
scratch bytes per lane, occupancy (waves / SIMD) and static LDS. Usage::

    python tools/kernel_resources.py csrc/kernels/ppo_rc.hip csrc/kernels/rollout.hip
"""

from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def analyse(src: str):
    inc = [f"-I{os.path.join(ROOT, 'csrc', d)}" for d in ("include", "kernels", "runtime")]
    cmd = [os.path.join(ROCM, "bin", "hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
           "--cuda-device-only", "-c", "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage", *inc, src]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(proc.stderr[-2000:])
    rows, cur = [], None
    for line in proc.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except OSError:
        return names


def main(srcs):
    print("| source | kernel instance | VGPR | AGPR | SGPR | scratch B/lane | waves/SIMD | LDS B |")
    print("|---|---|---|---|---|---|---|---|")
    for src in srcs:
        rows = analyse(src)
        names = demangle([r["name"] for r in rows])
        for r, n in zip(rows, names):
            n = re.sub(r"\(anonymous namespace\)::", "", n)
            n = n.split("(")[0] if "(" in n else n
            print(f"| {os.path.basename(src)} | `{n}` | {r.get('VGPRs', '?')} | {r.get('AGPRs', '?')} | {r.get('TotalSGPRs', '?')} | "
                  f"{r.get('ScratchSize [bytes/lane]', '?')} | {r.get('Occupancy [waves/SIMD]', '?')} | {r.get('LDS Size [bytes/block]', '?')} |")


if __name__ == "__main__":
    main(sys.argv[1:] or [os.path.join(ROOT, "csrc", "kernels", "ppo_rc.hip")])

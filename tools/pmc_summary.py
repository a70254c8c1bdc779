"""Per-kernel summary of a rocprofv3 --pmc CSV (counter_collection.csv): mean counter
values per dispatch, with derived per-wave instruction mix and the wait fraction."""
import sys

import pandas as pd

df = pd.read_csv(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
df["kernel"] = df["Kernel_Name"].str.slice(0, 70)
piv = df.pivot_table(index=["Dispatch_Id", "kernel", "Grid_Size", "Workgroup_Size", "VGPR_Count", "LDS_Block_Size"],
                     columns="Counter_Name", values="Counter_Value", aggfunc="sum").reset_index()
dur = df.groupby("Dispatch_Id").agg(t0=("Start_Timestamp", "min"), t1=("End_Timestamp", "max"))
piv = piv.merge(dur, left_on="Dispatch_Id", right_index=True)
piv["us"] = (piv["t1"] - piv["t0"]) / 1e3
g = piv.groupby(["kernel", "Grid_Size", "Workgroup_Size", "VGPR_Count", "LDS_Block_Size"]).mean(numeric_only=True)
g["calls"] = piv.groupby(["kernel", "Grid_Size", "Workgroup_Size", "VGPR_Count", "LDS_Block_Size"]).size()
g = g.sort_values("us", ascending=False).head(top)
print("| kernel | grid | wg | vgpr | lds B | calls | us/call | waves | VALU/wave | MFMA/wave | LDS/wave | SALU/wave | VMEM/wave | wait-any / busy |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
for k, r in g.iterrows():
    w = max(r.get("SQ_WAVES", 1), 1)
    ratio = r.get("SQ_WAIT_INST_ANY", 0) / max(r.get("SQ_BUSY_CYCLES", 1), 1)
    print(f"| `{k[0]}` | {k[1]} | {k[2]} | {k[3]} | {k[4]} | {int(r['calls'])} | {r['us']:.1f} | {w:.0f} | "
          f"{r.get('SQ_INSTS_VALU', 0) / w:.0f} | {r.get('SQ_INSTS_MFMA', 0) / w:.0f} | {r.get('SQ_INSTS_LDS', 0) / w:.0f} | "
          f"{r.get('SQ_INSTS_SALU', 0) / w:.0f} | {r.get('SQ_INSTS_VMEM', 0) / w:.0f} | {ratio:.2f} |")

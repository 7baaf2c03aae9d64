"""Summarise a rocprofv3 kernel trace CSV: per-kernel-name total/avg time and launch stats."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
agg = defaultdict(lambda: [0, 0.0, None])
for x in rows:
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    name = x["Kernel_Name"].split("(")[0][:70]
    a = agg[name]
    a[0] += 1
    a[1] += d
    a[2] = (x["VGPR_Count"], x["Accum_VGPR_Count"], x["SGPR_Count"], x["LDS_Block_Size"], x["Scratch_Size"], x["Grid_Size_X"])
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':70s} {'calls':>6s} {'total ms':>9s} {'avg ms':>8s} {'%':>6s}  vgpr/agpr/sgpr/lds/scratch/grid")
for k, (c, t, meta) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:70s} {c:6d} {t:9.3f} {t / c:8.4f} {100 * t / tot:6.2f}  {'/'.join(meta)}")
print(f"total kernel time {tot:.3f} ms over {len(rows)} dispatches")

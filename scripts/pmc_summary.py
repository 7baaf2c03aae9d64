"""Per-kernel per-wave PMC summary of a rocprofv3 --pmc counter_collection.csv (grouped by kernel + grid)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    key = (r["Kernel_Name"][:48], r["Grid_Size"], r.get("LDS_Block_Size", ""), r.get("VGPR_Count", ""))
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r["Dispatch_Id"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = v.get("SQ_WAVES", 0) or 1
    vals = " ".join(f"{c.replace('SQ_', '')}={x / w:.1f}" for c, x in sorted(v.items()) if c != "SQ_WAVES")
    print(f"{k[0]} grid={k[1]} lds={k[2]} vgpr={k[3]} dispatches={len(disp[k])} waves={w:.0f}: {vals}")

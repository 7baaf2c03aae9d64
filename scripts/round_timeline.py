"""Per-round GPU timeline of a bench run from a rocprofv3 kernel trace: rounds are delimited by the round
epilogue kernel (qfx_round_apply_kernel); prints, averaged over the last rounds, the round period, the kernel
busy time, the idle gaps between kernels and each kernel's average duration.

python scripts/round_timeline.py gpurun_out/prof/bench_kernel_trace.csv [--rounds 8]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--marker", default="qfx_round_apply_kernel")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    if len(ends) < 2:
        raise SystemExit("fewer than two round markers in the trace")
    sel = ends[-(args.rounds + 1):]
    per = defaultdict(float)
    cnt = defaultdict(int)
    period = busy = 0.0
    n = len(sel) - 1
    for a, b in zip(sel, sel[1:]):
        seg = rows[a + 1: b + 1]
        period += (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            busy += d
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            per[name] += d
            cnt[name] += 1
    print(f"rounds {n}: period {period / n:.1f} us, kernel busy {busy / n:.1f} us, idle {(period - busy) / n:.1f} us, "
          f"{sum(cnt.values()) / n:.1f} dispatches/round")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {k:60s} {cnt[k] / n:5.1f} x {v / cnt[k]:8.1f} us = {v / n:8.1f} us/round")


if __name__ == "__main__":
    main()

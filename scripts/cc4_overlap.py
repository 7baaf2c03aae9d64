"""CC4 evidence from a rocprofv3 kernel trace of a bench run with QFEDX_CC4=1 (one-rank RCCL group): every
side-stream upload + gather launch (qfx_round_prologue_kernel on a queue other than the round graph's) and the
main-queue kernels it ran concurrently with - the previous round's passes, reduction and collective - with the
overlapped microseconds.  Without CC4 the prologue sits on the graph's queue, in line with the passes.

python scripts/cc4_overlap.py gpurun_out/prof_cc4/..._kernel_trace.csv [--rounds 8]
"""
import argparse
import csv
from collections import Counter


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").split("<")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--rounds", type=int, default=8)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    qkey = next((k for k in ("Queue_Id", "Stream_Id", "Queue_ID") if k in rows[0]), None)
    if qkey is None:
        raise SystemExit(f"no queue column in {list(rows[0])}")

    def span(r):
        return int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    main_q = Counter(r[qkey] for r in rows if "hea_adj_kernel" in r["Kernel_Name"]).most_common(1)[0][0]
    side = [r for r in rows if "qfx_round_prologue_kernel" in r["Kernel_Name"] and r[qkey] != main_q]
    mains = [r for r in rows if r[qkey] == main_q]
    inline = sum(1 for r in mains if "qfx_round_prologue_kernel" in r["Kernel_Name"])
    print(f"round-graph queue {main_q}: {len(mains)} kernels ({inline} round prologues in line); "
          f"side-queue prologues (upload + gather): {len(side)}")
    for p in side[-args.rounds:]:
        p0, p1 = span(p)
        ov = []
        for m in mains:
            m0, m1 = span(m)
            o = min(p1, m1) - max(p0, m0)
            if o > 0:
                ov.append(f"{short(m['Kernel_Name'])} {o / 1e3:.1f}")
        print(f"  side prologue q{p[qkey]} {(p1 - p0) / 1e3:6.1f} us | concurrent with: {', '.join(ov) or 'nothing'}")
    colls = [r for r in mains + side if "nccl" in r["Kernel_Name"].lower() or "rccl" in r["Kernel_Name"].lower()]
    if colls:
        d = [(span(c)[1] - span(c)[0]) / 1e3 for c in colls[-args.rounds:]]
        print(f"collective kernels: {len(colls)}, last {len(d)} mean {sum(d) / len(d):.1f} us "
              f"({short(colls[-1]['Kernel_Name'])})")


if __name__ == "__main__":
    main()

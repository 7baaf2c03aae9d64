"""Split a rocprofv3 kernel trace of scripts/graph_gap.py into in-graph kernel time and inter-graph gaps.

python scripts/gap_split.py TRACE.csv KERNELS_PER_GRAPH
"""
import csv
import statistics
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "elementwise" in r["Kernel_Name"]]
    n = int(sys.argv[2])
    gaps, inner, dur = [], [], []
    for i in range(1, len(rows)):
        g = (int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3
        (gaps if i % n == 0 else inner).append(g)
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    med = statistics.median
    print(f"kernels {len(rows)}: median duration {med(dur):.2f} us, in-graph gap {med(inner) if inner else 0:.2f} us,"
          f" boundary gap median {med(gaps):.2f} us (p10 {sorted(gaps)[len(gaps) // 10]:.2f})")


if __name__ == "__main__":
    main()

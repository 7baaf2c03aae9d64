"""Per-round periods and pass-kernel durations, in launch order, from a rocprofv3 kernel trace of bench.py.

python scripts/round_periods.py <kernel_trace.csv>   (a round starts at each qfx_round_prologue_kernel)
"""
import csv
import sys


def main(path):
    r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    starts = [int(x["Start_Timestamp"]) for x in r if "prologue" in x["Kernel_Name"]]

    def durs(tag):
        return [(int(x["Start_Timestamp"]), (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
                for x in r if tag in x["Kernel_Name"]]
    adj, fwd = durs("hea_adj"), durs("hea_fwd")
    print("round  period_us  fwd_us(2)  adj_us(2)")
    for i in range(len(starts) - 1):
        a = [d for s, d in adj if starts[i] <= s < starts[i + 1]]
        f = [d for s, d in fwd if starts[i] <= s < starts[i + 1]]
        print(f"{i:5d} {(starts[i + 1] - starts[i]) / 1e3:10.1f}  {' '.join(str(round(x)) for x in f):>9s}  "
              f"{' '.join(str(round(x)) for x in a):>9s}")


if __name__ == "__main__":
    main(sys.argv[1])

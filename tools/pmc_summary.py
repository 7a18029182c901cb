"""Sum rocprofv3 --pmc counter_collection CSVs over one kernel's dispatches, per fold.

usage: python tools/pmc_summary.py FOLDS CSV [CSV ...] [KERNEL]
level_profile.py runs FOLDS=2 folds; every counter is summed over all dispatches of the matched
kernel (default k_level4d) and divided by FOLDS.  Also prints the average dispatch duration.
"""
import csv
import sys
from collections import defaultdict


def main(argv):
    folds = float(argv[1])
    kern = "k_level4d"
    if argv and not argv[-1].endswith(".csv"):
        kern = argv.pop()
    tot = defaultdict(float)
    dur = {}
    for path in argv[2:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                if not r["Kernel_Name"].replace("void ", "", 1).startswith(kern):
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                dur[(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k in sorted(tot):
        print(f"{k} {tot[k] / folds:.6g}")
    if dur:
        print(f"dispatches {len(dur)} avg_us {sum(dur.values()) / len(dur) / 1e3:.1f}")


if __name__ == "__main__":
    main(sys.argv)

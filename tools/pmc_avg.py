"""Average rocprofv3 --pmc counters per dispatch of kernels matching a regex (development tool).
usage: pmc_avg.py <dir with *_counter_collection.csv> <kernel regex>"""
import collections
import csv
import glob
import re
import sys


def main():
    d, kre = sys.argv[1:3]
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if re.search(kre, r["Kernel_Name"]):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{d} {k} {sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main()

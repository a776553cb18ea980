"""Average rocprofv3 counter_collection.csv values per counter for one kernel
(name substring), over all its dispatches: python tools/pmc_summary.py DIR [KERNEL]"""
import collections
import csv
import glob
import sys


def summary(d, kern="gemm"):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    s = summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "gemm")
    for k in sorted(s):
        print(f"{k:32s} {s[k]:16.4g}")

"""Shorten a rocprofv3 ``--stats`` kernel CSV (run_kernel_stats.csv) into the
table committed under profiles/.  Usage:

  python tools/stats_summary.py <run_kernel_stats.csv> "<header line>" [top]
"""
import csv
import re
import subprocess
import sys


def short(name: str) -> str:
    if name.startswith("_Z"):
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True,
                                  check=True).stdout.strip()
        except Exception:
            pass
    if name.startswith("_Z"):   # c++filt lacks the bf16 (DF16b) mangling
        k = re.search(r"N_1\d+(\w+?_kernel)", name)
        op = re.search(r"ENS0_\d+(\w+?Op)I", name)
        name = "dcnr::" + (k.group(1) if k else name[:60]) + "<bf16" + \
            (", " + op.group(1) if op else "") + ">"
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*\)$", "", name)
    return name[:110]


def main():
    path, header = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(header)
    print()
    print(f"{'total_ms':>9} {'calls':>6} {'avg_us':>9} {'pct':>6}  kernel")
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e6:9.2f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{100 * t / tot:6.2f}  {short(r['Name'])}")
    print(f"{tot / 1e6:9.2f} total kernel time (ms)")


if __name__ == "__main__":
    main()

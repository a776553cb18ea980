"""Per-call timeline of the fused eval forward from a rocprofv3 trace of
tools/tower_probe.py (kernel trace, and the memory-copy trace if present):
for consecutive tower_kernel calls, the kernels and copies between the end
of one tower launch and the end of the next, with the idle gaps.

  python tools/eval_timeline.py <dir with *_kernel_trace.csv> [--calls 3]
"""
import argparse
import csv
import glob
import re


def load(d):
    ev = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(anonymous namespace\)::|dcnr::|void ", "", r["Kernel_Name"]).split("(")[0][:50]
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "copy " + r.get("Direction", "") + " " + r.get("Bytes", "")))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    ev = load(a.dir)
    tw = [i for i, e in enumerate(ev) if "tower_kernel" in e[2]]
    # calls in the middle of the run
    mid = len(tw) // 2
    tot_gap, n = 0.0, 0
    for j in range(mid, min(mid + a.calls, len(tw) - 1)):
        i0, i1 = tw[j], tw[j + 1]
        base = ev[i0][1]
        print(f"call {j}: {(ev[i1][1] - base) / 1e3:.1f} us from tower end to tower end")
        last = base
        for s, e, name in ev[i0 + 1:i1 + 1]:
            gap = (s - last) / 1e3
            print(f"   gap {gap:7.1f}   {(s - base) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {name}")
            if gap > 0:
                tot_gap += gap
            last = max(last, e)
        n += 1
    if n:
        print(f"mean idle per call: {tot_gap / n:.1f} us")


if __name__ == "__main__":
    main()

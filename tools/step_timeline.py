"""One train step's kernel timeline from a rocprofv3 kernel trace of bench.py.

Picks the step that ends with the N-th `adam_kernel` dispatch (default: the
middle of the plain timed pass), lists every kernel that starts inside it by
start time with its queue, and sums the idle gaps of the main queue (the
queue adam runs on) -- where the step waits on cross-stream events.

  python tools/step_timeline.py run_kernel_trace.csv --step 12 [--all]
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=12, help="index of the adam dispatch ending the step")
    ap.add_argument("--all", action="store_true", help="print every kernel, not only the gaps")
    ap.add_argument("--min-gap", type=float, default=3.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    for r in rows:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["t0"])
    adam = [r for r in rows if "adam_kernel" in r["Kernel_Name"]]
    end, prev = adam[a.step], adam[a.step - 1]
    main_q = end[qkey]
    step = [r for r in rows if prev["t1"] <= r["t0"] <= end["t1"]]
    base = prev["t1"]
    gaps, last_end = [], base
    print(f"step {a.step}: {(end['t1'] - base) / 1e3:.1f} us, {len(step)} kernels, main queue {main_q}")
    for r in step:
        name = re.sub(r"\(anonymous namespace\)::|dcnr::|void ", "", r["Kernel_Name"]).split("(")[0][:60]
        on_main = r[qkey] == main_q
        if on_main:
            g = (r["t0"] - last_end) / 1e3
            if g >= a.min_gap:
                gaps.append((g, name))
            last_end = max(last_end, r["t1"])
        if a.all:
            print(f"{(r['t0'] - base) / 1e3:9.1f} {(r['t1'] - r['t0']) / 1e3:8.1f} "
                  f"{'M' if on_main else 'S'}{r[qkey]:>3} {name}")
    tot = sum(g for g, _ in gaps)
    print(f"main-queue gaps >= {a.min_gap} us: {len(gaps)}, {tot:.1f} us")
    for g, n in gaps:
        print(f"  {g:7.1f} us before {n}")


if __name__ == "__main__":
    main()

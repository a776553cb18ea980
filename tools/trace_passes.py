"""Per-pass averages of one kernel from a rocprofv3 kernel trace of bench.py.

bench.py times K plain steps (the reported value), then the same K steps
with every launch bracketed by HIP events (the roofline pass).  In the plain
pass the bf16 weight-gradient GEMMs run on the side stream, concurrently
with the main stream's dX GEMMs and BN passes; in the instrumented pass the
library runs them alone on the main stream.  rocprofv3 --stats averages over
both, so this splits the kernel's dispatches (in dispatch order) into
[warmup | plain | instrumented] by the per-step launch count.

  python tools/trace_passes.py run_kernel_trace.csv gemm_dw_kernel \
      --per-step 9 --warmup 5 --steps 20
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("--per-step", type=int, required=True)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    w, k = a.warmup * a.per_step, a.steps * a.per_step
    legs = {"warmup": dur[:w], "plain (side stream, concurrent)": dur[w:w + k],
            "instrumented (alone, main stream)": dur[w + k:w + 2 * k]}
    print(f"{a.kernel}: {len(dur)} dispatches")
    for name, d in legs.items():
        if d:
            print(f"  {name:36s} n={len(d):4d} avg_us={sum(d) / len(d):8.2f} "
                  f"min_us={min(d):8.2f} max_us={max(d):8.2f}")


if __name__ == "__main__":
    main()

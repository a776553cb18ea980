"""Per-step HBM ledger: every dispatch of ONE train step with its PMC bytes,
then per kernel class the PMC bytes against the library's algorithmic bytes.

The PMC passes (tools/profile_round.sh: FETCH_SIZE and WRITE_SIZE, separate
runs, dispatches serialised by the profiler) see every dispatch of the run;
the step is the dispatches after the (N-1)-th `adam_kernel` up to the N-th.
FETCH_SIZE is doubled on gfx950, WRITE_SIZE taken as is (MI355X_MICROARCH.md,
HBM section; the same corrections as tools/pmc_traffic.py).  Algorithmic
bytes per class come from the bench JSON line of a run of the same tree
(`roofline_by_class[*].bytes_per_launch` x `launches_per_step`: inputs read
once, outputs written once, counted by the library at each launch).

  python tools/pmc_ledger.py <fetch csv> <write csv> [--bench bench.log] [--step 3]
"""
import argparse
import csv
import json
import re
from collections import OrderedDict

# kernel-name pattern -> the library's kernel classes (bench.py roofline_by_class)
CLASSES = [
    ("gather_cross", r"gather_lowrank_kernel|gather_cross_v4_kernel|gather_cross_fwd"),
    ("gemm_fwd", r"gemm_wsp_kernel|gemm_ws_kernel<16, [03](, (\d|true|false))?>"),
    ("gemm_dx", r"gemm_ws_kernel<16, [12459](, (\d|true|false))?>"),
    ("gemm_dw", r"gemm_dw_kernel"),
    ("rowwise", r"rowcol_kernel"),
    ("reduce", r"reduce_small_kernel|reduce_fused_kernel|splitk_reduce_t_kernel|bce_final"),
    ("cross_bwd", r"cross_gram|cross_coef|cross_scalar|x0_alpha|cross_final"),
    ("emb_sort", r"emb_ids|emb_hist|emb_scan|emb_scatter|emb_bucket"),
    ("emb_sum", r"emb_runs"),
    ("adam", r"adam_kernel"),
]


def short(name):
    name = re.sub(r"\(anonymous namespace\)::|dcnr::|void ", "", name)
    name = re.sub(r"\(.*", "", name)
    name = name.replace("_ZN4dcnr12_GLOBAL__N_1", "")
    return name[:64]


def cls_of(name):
    for c, pat in CLASSES:
        if re.search(pat, name):
            return c
    return "other"


def load(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def step_rows(rows, step):
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    return rows[adam[step - 1] + 1: adam[step] + 1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--bench", help="bench.py log whose last line is the JSON result")
    ap.add_argument("--step", type=int, default=3, help="the step ending with this adam dispatch")
    a = ap.parse_args()
    fe = step_rows(load(a.fetch, "FETCH_SIZE"), a.step)
    wr = step_rows(load(a.write, "WRITE_SIZE"), a.step)
    if [short(r["Kernel_Name"]) for r in fe] != [short(r["Kernel_Name"]) for r in wr]:
        raise SystemExit("the two passes' steps differ in their dispatch sequence")
    phase = "fwd"
    per = OrderedDict()
    tot = {"fwd": [0.0, 0.0], "bwd": [0.0, 0.0], "opt": [0.0, 0.0]}
    print(f"{'#':>3} {'ph':3} {'read_MB':>9} {'write_MB':>9}  kernel")
    for i, (f, w) in enumerate(zip(fe, wr)):
        name = f["Kernel_Name"]
        rb = 2.0 * float(f["Counter_Value"]) * 1024.0
        wb = float(w["Counter_Value"]) * 1024.0
        if "adam_kernel" in name:
            phase = "opt"
        print(f"{i:3d} {phase:3} {rb / 1e6:9.2f} {wb / 1e6:9.2f}  {short(name)}")
        tot[phase][0] += rb
        tot[phase][1] += wb
        c = cls_of(name)
        e = per.setdefault(c, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += rb
        e[2] += wb
        if "bce_final" in name:
            phase = "bwd"
    print()
    for ph, (rb, wb) in tot.items():
        print(f"{ph}: read {rb / 1e9:.3f} GB  write {wb / 1e9:.3f} GB  total {(rb + wb) / 1e9:.3f} GB")
    alg = {}
    if a.bench:
        lines = [ln for ln in open(a.bench).read().splitlines() if ln.startswith("{")]
        for c, v in (json.loads(lines[-1]) if lines else {}).get("roofline_by_class", {}).items():
            alg[c] = v["bytes_per_launch"] * v["launches_per_step"]
    print()
    print(f"{'class':14} {'launches':>8} {'PMC_MB':>9} {'alg_MB':>9} {'PMC/alg':>8}")
    for c, (n, rb, wb) in sorted(per.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
        al = alg.get(c)
        ratio = f"{(rb + wb) / al:8.2f}" if al else f"{'':8}"
        als = f"{al / 1e6:9.1f}" if al else f"{'':9}"
        print(f"{c:14} {n:8d} {(rb + wb) / 1e6:9.1f} {als} {ratio}")


if __name__ == "__main__":
    main()

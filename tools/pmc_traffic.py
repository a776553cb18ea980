"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Follows MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE need
separate passes; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled; WRITE_SIZE is exact for 16-B stores and
float atomics.  Both counters are in KB.  Usage:

  python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> \
      [--json profiles/pmc_traffic.json]
"""
import argparse
import csv
import json
import re
from collections import defaultdict

# libdcnr kernel-name patterns (regular expressions) -> the bench's kernel classes
CLASSES = [
    # deep-tower forward Linears: initial layer (EPI 0) + 8 BN-input layers (EPI 3)
    # (template args <KTP, EPI, HB>: HB = 1-bit keep masks)
    ("gemm_fwd", r"gemm_wsp_kernel|gemm_ws_kernel<16, [03](, (\d|true|false))?>"),
    ("gemm_dx_bn", r"gemm_ws_kernel<16, [45](, (\d|true|false))?>"),
    ("gemm_resid", r"gemm_ws_kernel<16, [29](, (\d|true|false))?>"),
    ("gemm_f32", r"gemm_ws_kernel<16, 1(, (\d|true|false))?>"),
    ("gemm_eval_bn", r"gemm_ws_kernel<16, [67](, (\d|true|false))?>"),
    ("gemm_dw", r"gemm_dw_kernel"),
    ("gather_cross", r"gather_lowrank_kernel|gather_cross_fwd_kernel|gather_cross_v4_kernel<\d, \d, \d, 1>"),
    ("gather_cross_cfg2", r"gather_cross_v4_kernel<\d, \d, \d, 0>"),
    ("cross_bwd", r"cross_bwd(_v4)?_kernel"),
    ("adam", r"adam_kernel"),
]


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)
    return name[:110]


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--json")
    a = ap.parse_args()
    fe = load(a.fetch, "FETCH_SIZE")
    wr = load(a.write, "WRITE_SIZE")
    rows = []
    for name in sorted(set(fe) | set(wr)):
        f = fe.get(name, [])
        w = wr.get(name, [])
        fb = 2.0 * sum(f) / len(f) if f else 0.0
        wb = sum(w) / len(w) if w else 0.0
        rows.append((name, len(f), fb, wb))
    rows.sort(key=lambda r: -(r[2] + r[3]) * r[1])
    print(f"{'launches':>8} {'read_MB':>10} {'write_MB':>10}  kernel (per-launch HBM bytes; "
          f"FETCH_SIZE x2, WRITE_SIZE x1)")
    for name, n, fb, wb in rows:
        print(f"{n:8d} {fb / 1e6:10.2f} {wb / 1e6:10.2f}  {short(name)}")
    out = {}
    for cls, pat in CLASSES:
        sel = [r for r in rows if re.search(pat, r[0])]
        if sel:
            n = sum(r[1] for r in sel)
            out[cls] = sum((r[2] + r[3]) * r[1] for r in sel) / max(n, 1)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

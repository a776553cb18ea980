"""Per-kernel SQ counter summary from tools/sq_counters.sh's PMC passes.

  python tools/sq_summary.py <dir with p1/ p2/ counter_collection.csv files>

Counter units (MI355X_MICROARCH.md, "Per-instruction cycle constants"):
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over
waves; SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles the matrix pipe is busy
(16 per v_mfma_f32_16x16x32_bf16), summed over the 1024 SIMDs;
GRBM_GUI_ACTIVE is GPU-busy cycles summed over the 8 XCDs.  So per dispatch:

  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)
  clock_GHz = GRBM_GUI_ACTIVE / 8 / duration
  lds_wait  = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES   (waves stalled issuing LDS)
  bank_conf = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import glob
import re
import sys

GROUPS = [
    ("gemm_wsp<0,0> fwd BIAS (pipelined)", r"gemm_wsp_kernel<false, false>"),
    ("gemm_wsp<1,0> fwd BIAS_STATS (pipelined)", r"gemm_wsp_kernel<true, false>"),
    ("gemm_ws<16,0> fwd BIAS (initial Linear)", r"gemm_ws_kernel<16, 0>"),
    ("gemm_ws<16,3> fwd BIAS_STATS (BN inputs)", r"gemm_ws_kernel<16, 3>"),
    ("gemm_ws<16,4> dX RESID_BN", r"gemm_ws_kernel<16, 4>"),
    ("gemm_ws<16,5> dX DROP_BN", r"gemm_ws_kernel<16, 5>"),
    ("gemm_ws<16,2> dX RESID", r"gemm_ws_kernel<16, 2>"),
    ("gemm_ws<16,1> dX0 F32", r"gemm_ws_kernel<16, 1>"),
    ("gemm_ws<16,6/7> eval BN_RELU", r"gemm_ws_kernel<16, [67]>"),
    ("gemm_dw", r"gemm_dw_kernel"),
    ("splitk_reduce", r"splitk_reduce"),
    ("rowcol (BN row passes)", r"rowcol"),
    ("reduce_fused (BN finalize)", r"reduce_fused|reduce_small"),
    ("gather_cross", r"gather_cross"),
    ("emb_runs", r"emb_runs"),
    ("adam", r"adam_kernel"),
    ("knn scan4<2,16> (256 queries)", r"scan4_kernel<2, 16"),
    ("knn scan4<2,2> (<= 32 queries)", r"scan4_kernel<2, 2,"),
    ("knn rescore", r"rescore_kernel"),
    ("knn scan3", r"scan3_kernel"),
    ("tower_kernel (fused eval tower)", r"tower_kernel"),
    ("tower_pack", r"tower_pack"),
]


def demangle(names):
    import subprocess
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                             check=True).stdout.split("\n")
        return dict(zip(names, out))
    except Exception:
        return {n: n for n in names}


def load(d):
    # (dispatch id) -> {counter: value}, name, duration
    disp = collections.defaultdict(dict)
    meta = {}
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            key = (f.split("/p")[-1].split("/")[0], r.get("Dispatch_Id") or r.get("Correlation_Id"))
            disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            dur = None
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            meta[key] = (r["Kernel_Name"], dur)
    return disp, meta


def main():
    d = sys.argv[1]
    disp, meta = load(d)
    names = sorted({m[0] for m in meta.values()})
    dm = demangle(names)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, cs in disp.items():
        name, dur = meta[key]
        full = dm.get(name, name).replace("(anonymous namespace)::", "")
        g = next((g for g, pat in GROUPS if re.search(pat, full)), None)
        if g is None:
            continue
        for c, v in cs.items():
            per[g][c].append(v)
        if dur:
            per[g]["_dur_" + key[0]].append(dur)
    print("SQ counters per production kernel (averages per dispatch; bench.py --steps 2 "
          "--warmup 1 --eval-steps 1 under rocprofv3 --pmc, two passes)")
    print("mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8); "
          "lds_wait = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES; bank_conf = SQ_LDS_BANK_CONFLICT / "
          "SQ_LDS_IDX_ACTIVE; wait_any / active = SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES")
    print()
    hdr = f"{'kernel':42s} {'n':>3s} {'dur_us':>7s} {'GHz':>5s} {'mfma_busy':>9s} {'lds_wait':>8s} " \
          f"{'bank_conf':>9s} {'wait_any':>8s} {'active':>6s} {'lds_act':>7s} {'vmem_act':>8s} {'valu_act':>8s}"
    print(hdr)
    rows = {}
    for g, _ in GROUPS:
        if g not in per:
            continue
        c = {k: sum(v) / len(v) for k, v in per[g].items()}
        n = len(per[g].get("SQ_WAVE_CYCLES", per[g].get("SQ_LDS_IDX_ACTIVE", [])))
        dur = c.get("_dur_1") or c.get("_dur_2")
        grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        mb = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * grbm / 8) if grbm else float("nan")
        ghz = grbm / 8 / dur / 1e9 if (grbm and dur) else float("nan")
        lw = c.get("SQ_WAIT_INST_LDS", 0.0) / wc
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / (c.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0)
        wa = c.get("SQ_WAIT_ANY", 0.0) / wc
        ac = c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
        la = c.get("SQ_ACTIVE_INST_LDS", 0.0) / wc
        va = c.get("SQ_ACTIVE_INST_VMEM", 0.0) / wc
        vl = c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
        rows[g] = dict(c)
        print(f"{g:42s} {n:3d} {1e6 * (dur or 0):7.1f} {ghz:5.2f} {mb:9.3f} {lw:8.3f} {bc:9.3f} "
              f"{wa:8.3f} {ac:6.3f} {la:7.3f} {va:8.3f} {vl:8.3f}")
    print()
    print("raw averages per dispatch:")
    for g, c in rows.items():
        print(g)
        for k in sorted(c):
            if not k.startswith("_"):
                print(f"    {k:28s} {c[k]:16.6g}")


if __name__ == "__main__":
    main()

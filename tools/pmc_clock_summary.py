"""Summarise tools/pmc_clock.sh output dirs: per kernel, the median over its
dispatches of duration, effective clock (GRBM_GUI_ACTIVE / 8 / duration),
MFMA-busy (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) and
the wave-state split.  python tools/pmc_clock_summary.py DIR..."""
import collections
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    disp = collections.defaultdict(dict)
    meta = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Dispatch_Id") or r.get("Correlation_Id")
            disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 \
                if r.get("Start_Timestamp") else None
            meta[k] = (r["Kernel_Name"][:60], dur)
    rows = collections.defaultdict(list)
    for k, c in disp.items():
        name, dur = meta[k]
        g = c.get("GRBM_GUI_ACTIVE", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        rows[name].append((dur or 0.0, g / 8 / dur / 1e9 if dur and g else 0.0,
                           c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * g / 8) if g else 0.0,
                           c.get("SQ_WAIT_INST_ANY", 0.0) / wc, c.get("SQ_WAIT_ANY", 0.0) / wc,
                           c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc))
    for name, v in rows.items():
        med = [statistics.median(x) for x in zip(*v)]
        print(f"{d}: {name} n={len(v)} dur_us={med[0] * 1e6:.1f} GHz={med[1]:.2f} "
              f"mfma_busy={med[2]:.3f} wait_inst={med[3]:.3f} wait_any={med[4]:.3f} active={med[5]:.3f}")

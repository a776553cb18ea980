"""HBM bytes per launch of the kNN kernels, per (kernel, grid size), from two
rocprofv3 PMC passes over tools/knn_lab.py (FETCH_SIZE doubled on gfx950,
WRITE_SIZE exact; both in KB; MI355X_MICROARCH.md "HBM [CDNA4]"):
  python3 tools/knn_pmc.py <fetch run_counter_collection.csv> <write ...csv>"""
import csv
import re
import sys
from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        n = r["Kernel_Name"].replace("void ", "").replace("dcnr::(anonymous namespace)::", "")
        m = re.match(r"_ZN4dcnr12_GLOBAL__N_1(\d+)", n)
        if m:
            n = n[m.end():m.end() + int(m.group(1))]
        n = re.sub(r"\(.*", "", n)
        if not n.startswith(("kth", "bound5", "scan", "rescore", "merge")):
            continue
        per[(n, int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024.0)
    return per


fe, wr = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
print(f"{'launches':>8} {'read_MB':>9} {'write_MB':>9}  kernel [grid threads]")
for k in sorted(set(fe) | set(wr)):
    f, w = fe.get(k, []), wr.get(k, [])
    print(f"{len(f):8d} {2 * sum(f) / max(len(f), 1) / 1e6:9.2f} {sum(w) / max(len(w), 1) / 1e6:9.2f}  "
          f"{k[0]} [{k[1]}]")

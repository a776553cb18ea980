"""Per (kernel, grid) average durations of the kNN kernels in tools/knn_lab.sh runs:
  python3 tools/knn_lab_summary.py <outdir> v1 v2 ...   (first two calls of each skipped)"""
import csv, sys, re, collections
for v in sys.argv[2:]:
    rows = list(csv.DictReader(open(f"{sys.argv[1]}/{v}/run_kernel_trace.csv")))
    agg = collections.defaultdict(list)
    for r in rows:
        n = r['Kernel_Name'].replace('void ', '').replace('dcnr::(anonymous namespace)::', '')
        if not n.startswith(('scan4', 'rescore', 'bound5')): continue
        n = re.sub(r'\(.*', '', n)
        agg[(n, r['Grid_Size_X'], r['Grid_Size_Y'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    print(v, '  '.join('%s[%sx%s] %.1f' % (k[0], k[1], k[2], sum(t[2:]) / len(t[2:])) for k, t in sorted(agg.items())))

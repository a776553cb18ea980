"""Per-call breakdown of the kNN kernels in a rocprofv3 kernel trace of
tools/knn_probe.py: usage  python3 tools/knn_trace.py <run_kernel_trace.csv> [every]"""
import csv
import re
import sys

KN = ('kth', 'bound5', 'scan', 'rescore', 'merge', 'v4_prep')
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
every = int(sys.argv[2]) if len(sys.argv) > 2 else 13
seq = []
for r in rows:
    n = r['Kernel_Name'].replace('void ', '').replace('dcnr::(anonymous namespace)::', '')
    m = re.match(r'_ZN4dcnr12_GLOBAL__N_1(\d+)', n)   # left mangled by the tracer
    if m:
        n = n[m.end():m.end() + int(m.group(1))]
    if n.startswith(KN) or 'fillBuffer' in n:
        seq.append((re.sub(r'\(.*', '', n), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
                    r['Grid_Size_X'], r['Grid_Size_Y'], r['VGPR_Count'], int(r['Start_Timestamp'])))
calls, cur = [], []
for s in seq:
    if s[0].startswith(('kth', 'bound5')) and cur:
        calls.append(cur)
        cur = []
    cur.append(s)
calls.append(cur)
for i, c in enumerate(calls):
    if i % every != every - 1:
        continue
    t0 = c[0][5]
    print('--- call %d  span %.1f us' % (i, (c[-1][5] - t0) / 1e3 + c[-1][1]))
    for s in c:
        print('  %-34s %7.1f us  grid %s x %s  vgpr %s  start +%.1f' % (s[0][:34], s[1], s[2], s[3], s[4],
                                                                      (s[5] - t0) / 1e3))

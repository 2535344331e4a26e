"""Median kernel duration per (kernel, grid) from a rocprofv3 --kernel-trace CSV directory."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
d = defaultdict(list)
for r in csv.DictReader(open(f)):
    key = (r['Kernel_Name'].split('(')[0][:40], r.get('Grid_Size_X', r.get('Grid_Size', '')),
           r.get('Grid_Size_Y', ''), r.get('Grid_Size_Z', ''))
    d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items()):
    print(f'{k[0]:40s} grid {k[1]}x{k[2]}x{k[3]}  n={len(v)}  median {statistics.median(v):8.2f} us')

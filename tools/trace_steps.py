"""Kernel timeline of the bench's timed steps from a rocprofv3 --kernel-trace CSV: per kernel of
one step its duration and the gap since the previous kernel ended (graph replays back to back).
python tools/trace_steps.py DIR [kernels_per_step]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
f = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']),
              r['Kernel_Name'].split('(')[0].replace('void ', '')) for r in rows))
kd = [e for e in ev if 'kd::' in e[2]]
# the step starts at kd_prepare_fwd, or at kd_bin_count when the projection is inside the
# binning launch (the from-vertices node)
n_prep = sum('prepare_fwd' in e[2] for e in kd)
first = 'prepare_fwd' if n_prep >= sum('bin_count' in e[2] for e in kd) else 'bin_count'
starts = [i for i, e in enumerate(kd) if first in e[2]]
steps = [kd[a:b] for a, b in zip(starts, starts[1:])]
# the graph replays (back-to-back launches) are the steps with the shortest span; the eager
# profiling pass that follows them in bench.py has host-side gaps
steps = sorted(steps, key=lambda st: st[-1][1] - st[0][0])[:10]
agg = defaultdict(list)
tot = []
for st in steps:
    tot.append((st[-1][1] - st[0][0]) / 1e3)
    prev = None
    for k, (s, e, n) in enumerate(st):
        agg[(k, n)].append(((e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
        prev = e
print(f'steps {len(steps)}: first kernel start -> last kernel end {min(tot):.1f} / '
      f'{sorted(tot)[len(tot) // 2]:.1f} us (min / median)')
for (k, n), v in sorted(agg.items()):
    durs = sorted(x[0] for x in v)
    gaps = sorted(x[1] for x in v)
    print(f'  {k:2d} {n[:60]:60s} dur {durs[len(durs) // 2]:7.2f}  gap {gaps[len(gaps) // 2]:6.2f}')
# the period of consecutive steps in time order (the timed loop's replays are back to back: the
# shortest periods), and the gap between one step's last kernel and the next step's first
allst = [kd[a:b] for a, b in zip(starts, starts[1:])]
pairs = sorted(((allst[i + 1][0][0] - allst[i][0][0]) / 1e3,
                (allst[i + 1][0][0] - allst[i][-1][1]) / 1e3) for i in range(len(allst) - 1))
if pairs:
    best = pairs[:max(1, len(pairs) // 2)]
    print(f'step period (start to start, consecutive replays) median '
          f'{best[len(best) // 2][0]:.1f} us; gap between replays {best[len(best) // 2][1]:.1f} us')

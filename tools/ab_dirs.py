"""Same-box A/B of whole trees: python tools/ab_dirs.py DIR_A DIR_B [reps] [bench args...]

Runs DIR/bench.py (--no-cpu-baseline) alternately from each tree `reps` times and prints the best
median step time (ms_per_step_median) and per-kernel averages of each (box-to-box spread is a few %, so compare on one box)."""
import json
import os
import subprocess
import sys

dirs = [os.path.abspath(sys.argv[1]), os.path.abspath(sys.argv[2])]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
extra = sys.argv[4:]
res = {d: [] for d in dirs}
kern = {d: {} for d in dirs}
for r in range(reps):
    for d in dirs:
        p = subprocess.run([sys.executable, 'bench.py', '--no-cpu-baseline', '--steps', '40',
                            *extra], cwd=d, capture_output=True, text=True, timeout=600)
        lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
        if p.returncode != 0 or not lines:
            print(f'{d}: rc={p.returncode}\n{p.stderr[-2000:]}')
            sys.exit(1)
        out = json.loads(lines[-1])
        res[d].append(out.get('ms_per_step_median') or out['ms_per_step'])
        for k, v in out['kernels'].items():
            kern[d].setdefault(k, []).append(v['avg_us'])
        print(f'rep {r} {os.path.basename(d)}: {res[d][-1]:.4f} ms (median step)', flush=True)
for d in dirs:
    print(f'{os.path.basename(d)}: ms/step {sorted(res[d])}  best {min(res[d]):.4f}')
names = list(kern[dirs[0]]) + [k for k in kern[dirs[1]] if k not in kern[dirs[0]]]
for k in names:
    print(f'  {k:22s} ' + '  '.join(f'{min(kern[d].get(k, [0])):8.2f}' for d in dirs))

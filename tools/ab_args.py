"""Same-box A/B of two bench.py argument sets on this tree:
python tools/ab_args.py REPS "ARGS_A" "ARGS_B"   (e.g. 3 "--views-per-gpu 1" "--views-per-gpu 1
--vertex-bwd fused").  Runs them alternately and prints the median step times (ms_per_step_median)
and the per-kernel averages of each."""
import json
import os
import shlex
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps = int(sys.argv[1])
sets = [sys.argv[2], sys.argv[3]]
res = {a: [] for a in sets}
kern = {a: {} for a in sets}
for r in range(reps):
    for a in sets:
        p = subprocess.run([sys.executable, 'bench.py', '--no-cpu-baseline', '--steps', '40',
                            *shlex.split(a)], cwd=root, capture_output=True, text=True,
                           timeout=600)
        lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
        if p.returncode != 0 or not lines:
            print(f'[{a}]: rc={p.returncode}\n{p.stderr[-2000:]}')
            sys.exit(1)
        out = json.loads(lines[-1])
        res[a].append(out.get('ms_per_step_median') or out['ms_per_step'])
        for k, v in out['kernels'].items():
            kern[a].setdefault(k, []).append(v['avg_us'])
        print(f'rep {r} [{a}]: {res[a][-1]:.4f} ms (median step)', flush=True)
for a in sets:
    print(f'[{a}]: ms/step {sorted(res[a])}  best {min(res[a]):.4f}')
names = list(kern[sets[0]]) + [k for k in kern[sets[1]] if k not in kern[sets[0]]]
for k in names:
    print(f'  {k:22s} ' + '  '.join(f'{min(kern[a].get(k, [0])):8.2f}' for a in sets))

"""Same-box A/B of several trees: python tools/ab_multi.py reps DIR... [-- bench args]
Runs DIR/bench.py --no-cpu-baseline alternately and prints each tree's median step times and
per-kernel averages."""
import json
import os
import subprocess
import sys

args = sys.argv[1:]
extra = []
if '--' in args:
    extra = args[args.index('--') + 1:]
    args = args[:args.index('--')]
reps, dirs = int(args[0]), [os.path.abspath(d) for d in args[1:]]
res = {d: [] for d in dirs}
kern = {d: {} for d in dirs}
for r in range(reps):
    for d in dirs:
        p = subprocess.run([sys.executable, 'bench.py', '--no-cpu-baseline', '--steps', '100',
                            *extra], cwd=d, capture_output=True, text=True, timeout=600)
        lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
        if p.returncode != 0 or not lines:
            print(f'{d}: rc={p.returncode}\n{p.stderr[-2000:]}')
            sys.exit(1)
        out = json.loads(lines[-1])
        res[d].append(out.get('ms_per_step_median') or out['ms_per_step'])
        for k, v in out['kernels'].items():
            kern[d].setdefault(k, []).append(v['avg_us'])
        print(f'rep {r} {os.path.basename(d)}: {res[d][-1]:.4f} ms', flush=True)
for d in dirs:
    ks = ' '.join(f'{k}={sum(v) / len(v):.2f}' for k, v in kern[d].items())
    print(f'{os.path.basename(d)}: best {min(res[d]):.4f} all {sorted(res[d])} | {ks}')

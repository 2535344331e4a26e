"""Same-box A/B of one environment variable: python tools/ab_env.py NAME=VALUE [reps] [bench args]

Runs bench.py (--no-cpu-baseline --steps 40) alternately without and with NAME=VALUE and prints
each run's timed-loop ms_per_step and median per-step event time."""
import json
import os
import subprocess
import sys

name, _, value = sys.argv[1].partition('=')
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
extra = sys.argv[3:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {'off': [], 'on': []}
for r in range(reps):
    for tag in ('off', 'on'):
        env = dict(os.environ)
        env.pop(name, None)
        if tag == 'on':
            env[name] = value
        p = subprocess.run([sys.executable, 'bench.py', '--no-cpu-baseline', '--steps', '40', *extra],
                           cwd=root, env=env, capture_output=True, text=True, timeout=600)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
        if p.returncode != 0 or not lines:
            print(f'{tag}: rc={p.returncode}\n{p.stderr[-2000:]}')
            sys.exit(1)
        out = json.loads(lines[-1])
        res[tag].append((out['ms_per_step'], out.get('ms_per_step_median')))
        print(f'rep {r} {tag}: ms_per_step {out["ms_per_step"]:.4f}  median {out.get("ms_per_step_median")}',
              flush=True)
for tag in res:
    print(f'{name}={value if tag == "on" else "(unset)"}: best ms_per_step '
          f'{min(x[0] for x in res[tag]):.4f}, best median {min(x[1] for x in res[tag]):.4f}')

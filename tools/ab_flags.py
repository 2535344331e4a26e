"""Per-kernel eager times under diagnostic ablation flags (the diagnostic library):
python tools/ab_flags.py FLAGS [FLAGS ...] [-- bench args]   (FLAGS: ints, 0x.. allowed)

Each flag set runs bench.py --no-graph --no-cpu-baseline (KAOLIN_AMD_DIAG=1, KD_DEBUG_FLAGS) twice,
alternating, and prints the per-kernel HIP-event averages of the better run."""
import json
import os
import subprocess
import sys

argv = sys.argv[1:]
extra = argv[argv.index('--') + 1:] if '--' in argv else []
flags = argv[:argv.index('--')] if '--' in argv else argv
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
best = {}
for rep in range(2):
    for f in flags:
        env = dict(os.environ, KAOLIN_AMD_DIAG='1', KD_DEBUG_FLAGS=f)
        p = subprocess.run([sys.executable, 'bench.py', '--no-cpu-baseline', '--no-graph',
                            '--steps', '20', *extra], cwd=root, env=env, capture_output=True,
                           text=True, timeout=600)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
        if p.returncode != 0 or not lines:
            print(f'flags {f}: rc={p.returncode}\n{p.stderr[-1500:]}')
            sys.exit(1)
        k = {n: v['avg_us'] for n, v in json.loads(lines[-1])['kernels'].items()}
        b = best.setdefault(f, k)
        for n, v in k.items():
            b[n] = min(b.get(n, v), v)
names = sorted({n for k in best.values() for n in k})
print('kernel'.ljust(22) + ''.join(f'{f:>12s}' for f in flags))
for n in names:
    print(n.ljust(22) + ''.join(f'{best[f].get(n, 0):12.2f}' for f in flags))

"""A/B of kd_debug_set flags on the bench step time: python tools/ab_bench.py FLAGS_A FLAGS_B [reps]"""
import os
os.environ.setdefault('KAOLIN_AMD_DIAG', '1')  # the diagnostic build (ablation flags)
import subprocess
import sys
import json

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
a, b = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
code = ("import sys, runpy; sys.argv=['bench.py','--no-cpu-baseline','--steps','40']; "
        "from kaolin_amd import _lib; _lib.debug_set(%d); "
        "runpy.run_path('bench.py', run_name='__main__')")
res = {a: [], b: []}
kern = {a: {}, b: {}}
for r in range(reps):
    for f in (a, b):
        out = subprocess.run([sys.executable, '-c', code % f], cwd=root, capture_output=True,
                             text=True, timeout=600).stdout.strip().splitlines()[-1]
        d = json.loads(out)
        res[f].append(d['ms_per_step'])
        for k, v in d['kernels'].items():
            kern[f].setdefault(k, []).append(v['avg_us'])
for f in (a, b):
    print(f'flags={f}: ms/step {sorted(res[f])}  best {min(res[f]):.4f}')
for k in list(kern[a]) + [k for k in kern[b] if k not in kern[a]]:
    print(f'  {k:22s} ' + '  '.join(f'{f}: {min(kern[f].get(k, [0])):7.2f}' for f in (a, b)))

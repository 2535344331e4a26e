"""Per-kernel VGPR / scratch / LDS / occupancy of the gfx950 build (hipcc -Rpass-analysis)."""
import os
import re
import subprocess

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'kaolin_amd',
                    'csrc')
import sys
sys.path.insert(0, os.path.dirname(CSRC))
import _build  # noqa: E402  (the library's own flags: same code generation)

only = sys.argv[1:]
for f in sorted(x[:-4] for x in os.listdir(CSRC) if x.endswith('.hip')):
    if only and f not in only:
        continue
    out = subprocess.run(['/opt/rocm/bin/hipcc', *_build.FLAGS, *_build.SOURCE_FLAGS.get(f + '.hip', []),
                          '-c', f'{f}.hip', '-o', '/tmp/kd_ru.o',
                          '-Rpass-analysis=kernel-resource-usage'], cwd=CSRC,
                         capture_output=True, text=True).stderr
    cur = None
    for line in out.splitlines():
        m = re.search(r'Function Name: (\S+)', line)
        if m:
            cur = {'name': m.group(1)}
            continue
        for key, pat in (('vgpr', r'VGPRs: (\d+)'), ('scratch', r'ScratchSize \[bytes/lane\]: (\d+)'),
                         ('lds', r'LDS Size \[bytes/block\]: (\d+)'),
                         ('occ', r'Occupancy \[waves/SIMD\]: (\d+)'),
                         ('sspill', r'SGPRs Spill: (\d+)'), ('vspill', r'VGPRs Spill: (\d+)')):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = m.group(1)
        if cur and 'lds' in cur:  # the last field of a kernel's remark block
            print(f"{cur['name'][:64]:64s} vgpr={cur.get('vgpr')} scratch={cur.get('scratch')} "
                  f"lds={cur.get('lds')} occ={cur.get('occ')} "
                  f"spill(s/v)={cur.get('sspill')}/{cur.get('vspill')}")
            cur = None

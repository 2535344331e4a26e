#!/bin/bash
# Instruction counters of the bench step's kernels under diagnostic flags (KD_DEBUG_FLAGS): one
# rocprofv3 --pmc pass (SQ counters only) per flag value, eager launches.
# Usage: tools/pmc_flags.sh FLAGS...   (prints kernel: VALU / SALU / LDS instructions, waves)
cd /tmp && export TMPDIR=/tmp
export KAOLIN_AMD_DIAG=1  # the diagnostic build: device ablation switches
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$repo" || exit 2
mkdir -p gpurun_out
for f in "$@"; do
  d="gpurun_out/pmcf_$f"
  rm -rf "$d"
  KD_DEBUG_FLAGS=$f timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$d" -o run -- \
    python3 bench.py --no-cpu-baseline --no-graph --steps 3 --warmup 1 > "$d.log" 2>&1 || { echo "flags $f failed"; tail -3 "$d.log"; exit 1; }
  python3 - "$d" "$f" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0].replace('void kd::', '').replace('kd::', '')
    if not k.startswith('kd_'):
        continue
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[k].add(r['Dispatch_Id'])
for k, c in acc.items():
    m = len(n[k])
    print(f"flags {sys.argv[2]} {k[:26]:26s} VALU {c['SQ_INSTS_VALU']/m/1e6:7.2f}M SALU {c['SQ_INSTS_SALU']/m/1e6:7.2f}M LDS {c['SQ_INSTS_LDS']/m/1e6:6.2f}M waves {c['SQ_WAVES']/m:8.0f} cyc/wave {c['SQ_WAVE_CYCLES']/max(c['SQ_WAVES'],1):8.0f}", flush=True)
PY
done

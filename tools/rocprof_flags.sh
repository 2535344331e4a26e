#!/bin/bash
# Per-kernel rocprofv3 kernel-trace averages of the bench step under diagnostic flags
# (KD_DEBUG_FLAGS, kd_debug_set): one rocprof run per flag value, the summary of each printed.
# Usage: [TREE=dir] tools/rocprof_flags.sh FLAGS...   (bench of TREE, default the repo; extra bench
# args in $BENCH_ARGS).  Output under the repo's gpurun_out/.
cd /tmp && export TMPDIR=/tmp
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tree="${TREE:-$repo}"
tag=$(basename "$tree")
mkdir -p "$repo/gpurun_out"
cd "$tree" || exit 2
for f in "$@"; do
  d="$repo/gpurun_out/rpf_${tag}_$f"
  rm -rf "$d"
  KD_DEBUG_FLAGS=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 $BENCH_ARGS > "$d.log" 2>&1 || { echo "flags $f failed"; tail -5 "$d.log"; exit 1; }
  python3 - "$d" "$tag $f" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0])))
out = []
for r in rows:
    n = r['Name']
    if 'kd::' in n:
        out.append(f"{n.split('(')[0].replace('void kd::', '')[:28]}={float(r['AverageNs'])/1e3:.2f}")
print('tree/flags', sys.argv[2], ' '.join(out), flush=True)
PY
done

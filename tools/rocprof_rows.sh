#!/bin/bash
# Per-kernel rocprofv3 kernel-trace averages of tools/bench_rows.py for each tree given (A/B of
# variants made by tools/ab_variant.sh); KERNELS = substring filter (default kd_).
# Usage: tools/rocprof_rows.sh TREE...   Output under the repo's gpurun_out/.
cd /tmp && export TMPDIR=/tmp
repo="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$repo/gpurun_out"
for tree in "$@"; do
  tag=$(basename "$tree")
  d="$repo/gpurun_out/rows_$tag"
  rm -rf "$d"
  (cd "$repo/$tree" && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
    python3 tools/bench_rows.py --steps 20 > "$d.log" 2>&1) || { echo "tree $tree failed"; tail -5 "$d.log"; exit 1; }
  python3 - "$d" "$tag" "${KERNELS:-kd_}" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0])))
out = [f"{r['Name'].split('(')[0].replace('void kd::', '')[:24]}={float(r['AverageNs'])/1e3:.2f}"
       for r in rows if sys.argv[3] in r['Name']]
print('tree', sys.argv[2], ' '.join(out), flush=True)
PY
done

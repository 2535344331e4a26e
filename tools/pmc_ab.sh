#!/bin/bash
# Same-box instruction counts of two trees: the first PMC group of tools/pmc_run.sh (SQ_WAVES,
# SQ_INSTS_VALU / LDS / SALU, cycles and waits) for DIR_A and DIR_B, one rocprofv3 pass each.
# Usage: tools/pmc_ab.sh DIR_A DIR_B [bench args...]
a=$1; b=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
root=$PWD
grp="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for d in "$a" "$b"; do
  name=$(basename "$(cd "$d" && pwd)")
  out="$root/gpurun_out/pmc_ab_$name"
  rm -rf "$out" && mkdir -p "$out"
  (cd "$d" && timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p1" -o run -- \
     python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --no-graph "$@" > "$out/p1.log" 2>&1)
  rc=$?
  if [ $rc -ne 0 ]; then tail -5 "$out/p1.log"; exit $rc; fi
  echo "== $name"
  python3 "$root/tools/pmc_summary.py" "$out" | grep -A9 "dibr_fwd\|dibr_bwd\|bin_count"
done

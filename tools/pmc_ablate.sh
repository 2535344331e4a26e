#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_LDS / SQ_INSTS_SALU / SQ_WAIT_INST_ANY per kernel under diagnostic
# ablation flags (kd_debug_set; KD_DEBUG_FLAGS), one rocprofv3 pass per flag set.
# Usage: tools/pmc_ablate.sh OUTDIR FLAGS...   (e.g. 0x4000000 0x4000010)
out=${1:-gpurun_out/abl}; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p "$out"
for f in "$@"; do
  KD_DEBUG_FLAGS=$f timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d "$out/f$f" -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --no-graph > "$out/f$f.log" 2>&1
  rc=$?
  echo "flags $f rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_summary.py "$out/f$f" > "$out/f$f.txt" || exit 1
done

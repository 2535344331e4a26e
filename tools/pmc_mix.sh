#!/bin/bash
# Per-type VALU instruction counts of the bench step's kernels (two rocprofv3 --pmc passes of 8 SQ
# counters each, eager launches), into the same OUTDIR as tools/pmc_run.sh so that
# tools/pmc_summary.py / make_traffic.py merge them.  Usage: tools/pmc_mix.sh OUTDIR [bench args]
out=${1:-gpurun_out/pmc}; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p "$out"
i=10
for grp in "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "mix pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
done

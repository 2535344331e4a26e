#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, then the PMC passes (tools/pmc_run.sh,
# eager launches: counters per dispatch) and their summary -> gpurun_out/prof, gpurun_out/pmc.
# Usage: tools/profile_c3.sh [extra bench args for the PMC passes]
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/prof gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1
bash tools/pmc_run.sh gpurun_out/pmc --steps 5 --warmup 2 --no-graph "$@"
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt

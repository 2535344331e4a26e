#!/bin/bash
# Runs "label:::seconds:::command" steps in order on the GPU box.  Any failing step ends the
# sequence (no further GPU work in this call): a failed test may hide a GPU fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  label="${step%%:::*}"; rest="${step#*:::}"; secs="${rest%%:::*}"; cmd="${rest#*:::}"
  echo "=== [$label] (limit ${secs}s) $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc"
  tail -n 25 "gpurun_out/$label.log"
  if [ $rc -ne 0 ]; then echo "=== stopping after [$label] (rc=$rc)"; exit $rc; fi
done

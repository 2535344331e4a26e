cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "cp1:::300:::python tools/concurrency_probe.py --tile-history 1" \
 "cp0:::300:::python tools/concurrency_probe.py --tile-history 0"

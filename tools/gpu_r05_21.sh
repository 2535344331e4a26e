cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "dtP:::200:::python tools/bench_rows.py --rows deftet" \
 "dtP2:::200:::python tools/bench_rows.py --rows deftet"

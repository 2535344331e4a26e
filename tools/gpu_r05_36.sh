cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tests:::900:::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "rows:::300:::python tools/bench_rows.py > gpurun_out/rows_zero.jsonl"

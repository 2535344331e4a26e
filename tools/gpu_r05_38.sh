cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tf3:::400:::python -u -m pytest tests/test_gpu_f3.py -x -q --timeout 120 --timeout-method thread" \
 "rows:::300:::python tools/bench_rows.py > gpurun_out/rows_final.jsonl"

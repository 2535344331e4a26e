cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tf2:::400:::python -u -m pytest tests/test_gpu_f2.py -x -q --timeout 120 --timeout-method thread" \
 "row:::200:::python tools/bench_rows.py --rows texture_mapping"

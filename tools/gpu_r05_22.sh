cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tf3:::400:::python -u -m pytest tests/test_gpu_f3.py tests/test_gpu_parity.py tests/test_gpu_vertices.py -x -q --timeout 120 --timeout-method thread" \
 "dtP:::200:::python tools/bench_rows.py --rows deftet" \
 "ab:::600:::python tools/ab_dirs.py ab/base . 3"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tp:::500:::python -u -m pytest tests/test_gpu_vertices.py tests/test_gpu_parity.py tests/test_gpu_graphed_step.py tests/test_gpu_step_oracle.py -x -q --timeout 300 --timeout-method thread" \
 "ab8:::400:::python tools/ab_dirs.py ab/cur . 3" \
 "ab1:::400:::python tools/ab_dirs.py ab/cur . 3 --views-per-gpu 1"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tb:::400:::python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_graphed_step.py -x -q --timeout 300 --timeout-method thread" \
 "ab8:::400:::python tools/ab_dirs.py ab/head . 3" \
 "ab1:::400:::python tools/ab_dirs.py ab/head . 3 --views-per-gpu 1"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tl:::500:::python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_parity.py tests/test_gpu_graphed_step.py tests/test_gpu_pools.py tests/test_gpu_split.py tests/test_gpu_breadth.py -x -q --timeout 300 --timeout-method thread" \
 "abl:::500:::python tools/ab_dirs.py ab/head ab/lists 3 --lists" \
 "abl2:::500:::python tools/ab_dirs.py ab/lists ab/lists2 3 --lists" \
 "ab8:::400:::python tools/ab_dirs.py ab/lists . 3" \
 "ab1:::400:::python tools/ab_dirs.py ab/lists . 3 --views-per-gpu 1" \
 "ab2:::400:::python tools/ab_dirs.py ab/lists . 3 --views-per-gpu 2"

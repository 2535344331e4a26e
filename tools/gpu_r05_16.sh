cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tl:::500:::python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_pools.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
 "abl:::600:::python tools/ab_dirs.py ab/cur . 3 --lists"

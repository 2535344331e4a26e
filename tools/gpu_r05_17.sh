cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tp:::500:::python -u -m pytest tests/test_gpu_pools.py tests/test_gpu_lists.py -x -q --timeout 300 --timeout-method thread"

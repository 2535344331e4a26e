cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tfine:::300:::python -u -m pytest tests/test_gpu_fine.py -x -v --timeout 120 --timeout-method thread" \
 "tall:::600:::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "ab8:::400:::python tools/ab_dirs.py ab/base . 3" \
 "ab1:::400:::python tools/ab_dirs.py ab/base . 3 --views-per-gpu 1" \
 "ab2:::400:::python tools/ab_dirs.py ab/base . 2 --views-per-gpu 2"

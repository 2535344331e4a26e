cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tq:::400:::python -u -m pytest tests/test_gpu_breadth.py tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
 "ab8:::400:::python tools/ab_dirs.py ab/base . 3" \
 "ab1:::400:::python tools/ab_dirs.py ab/base . 3 --views-per-gpu 1" \
 "flags:::300:::bash tools/pmc_flags.sh 0 16777216 2>&1 | grep -E 'dibr_fwd|dibr_bwd|failed'"

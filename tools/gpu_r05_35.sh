cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh "abm:::800:::python tools/ab_multi.py 3 ab/base ab/r3 ab/r4"

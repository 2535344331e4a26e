cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "ab:::700:::python tools/ab_dirs.py ab/base ab/sc8 3" \
 "ab1:::500:::python tools/ab_dirs.py ab/base ab/sc8 3 --views-per-gpu 1"

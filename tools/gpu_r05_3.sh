cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "flags:::600:::bash tools/pmc_flags.sh 0 16777216 16777220 16785412 16785414 2>&1 | grep -E 'dibr_fwd|failed'"

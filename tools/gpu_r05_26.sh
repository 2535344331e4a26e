cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do
 steps+=("new$r:::200:::python tools/bench_rows.py --rows deftet --dt-fwd")
 for v in head v_rank v_feat; do steps+=("$v$r:::200:::cd ab/$v && python tools/bench_rows.py --rows deftet --dt-fwd"); done
done
bash tools/gpu_steps.sh "${steps[@]}"

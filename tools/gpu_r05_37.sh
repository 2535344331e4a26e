cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do
 for v in head w1 w2; do steps+=("${v}_$r:::200:::cd ab/$v && python tools/bench_rows.py --rows deftet --dt-fwd"); done
done
bash tools/gpu_steps.sh "${steps[@]}"

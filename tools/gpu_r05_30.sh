cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do
 steps+=("t32_$r:::200:::python tools/bench_rows.py --rows texture_mapping")
 for v in tx16 tx20; do steps+=("${v}_$r:::200:::cd ab/$v && python tools/bench_rows.py --rows texture_mapping"); done
done
bash tools/gpu_steps.sh "${steps[@]}"

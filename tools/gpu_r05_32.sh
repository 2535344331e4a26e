cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do
 steps+=("cur_$r:::200:::python tools/bench_rows.py --rows deftet")
 steps+=("dtb8_$r:::200:::cd ab/dtb8 && python tools/bench_rows.py --rows deftet")
done
bash tools/gpu_steps.sh "${steps[@]}"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do
 steps+=("w1f_$r:::200:::python tools/bench_rows.py --rows deftet --dt-fwd")
 steps+=("w1b_$r:::200:::python tools/bench_rows.py --rows deftet")
 steps+=("w4f_$r:::200:::cd ab/head && python tools/bench_rows.py --rows deftet --dt-fwd")
 steps+=("w4b_$r:::200:::cd ab/head && python tools/bench_rows.py --rows deftet")
done
bash tools/gpu_steps.sh "${steps[@]}"

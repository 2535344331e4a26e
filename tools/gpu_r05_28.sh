cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do
 steps+=("fwd_$r:::200:::python tools/bench_rows.py --rows deftet --dt-fwd")
 steps+=("rev_$r:::200:::cd ab/rev && python tools/bench_rows.py --rows deftet --dt-fwd")
done
steps+=("hist:::200:::python tools/dt_list_hist.py > gpurun_out/dt_hist.txt")
bash tools/gpu_steps.sh "${steps[@]}"

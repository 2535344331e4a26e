cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=("tf3:::400:::python -u -m pytest tests/test_gpu_f3.py -x -q --timeout 120 --timeout-method thread")
for r in 1 2; do
 steps+=("new_$r:::200:::python tools/bench_rows.py --rows deftet --dt-fwd")
 steps+=("head_$r:::200:::cd ab/head && python tools/bench_rows.py --rows deftet --dt-fwd")
 steps+=("newb_$r:::200:::python tools/bench_rows.py --rows deftet")
 steps+=("headb_$r:::200:::cd ab/head && python tools/bench_rows.py --rows deftet")
done
bash tools/gpu_steps.sh "${steps[@]}"

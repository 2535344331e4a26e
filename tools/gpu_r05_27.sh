cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=("tf3:::400:::python -u -m pytest tests/test_gpu_f3.py -x -q --timeout 120 --timeout-method thread")
for r in 1 2; do
 steps+=("g2048_$r:::200:::python tools/bench_rows.py --rows deftet --dt-fwd")
 for v in head g4096; do steps+=("${v}_$r:::200:::cd ab/$v && python tools/bench_rows.py --rows deftet --dt-fwd"); done
done
bash tools/gpu_steps.sh "${steps[@]}"

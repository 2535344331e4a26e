cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tf3:::400:::python -u -m pytest tests/test_gpu_f3.py -x -q --timeout 120 --timeout-method thread" \
 "d0:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=0 python tools/bench_rows.py --rows deftet --dt-fwd" \
 "d26:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=0x4000000 python tools/bench_rows.py --rows deftet --dt-fwd" \
 "dP:::200:::python tools/bench_rows.py --rows deftet"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tf3:::400:::python -u -m pytest tests/test_gpu_f3.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
 "dtA:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=0 python tools/bench_rows.py --rows deftet" \
 "dtB:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=0x2000000 python tools/bench_rows.py --rows deftet" \
 "dtP:::200:::python tools/bench_rows.py --rows deftet" \
 "bn:::300:::python bench.py --steps 200 --warmup 20"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "dt0:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=0 python tools/bench_rows.py --rows deftet" \
 "dt128:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=128 python tools/bench_rows.py --rows deftet" \
 "dt27:::200:::KAOLIN_AMD_DIAG=1 KD_DEBUG_FLAGS=0x8000000 python tools/bench_rows.py --rows deftet"

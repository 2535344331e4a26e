cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=()
for r in 1 2; do for sp in 256 512 1024 2048; do
 steps+=("s${sp}_$r:::200:::cp ab/spans/lib$sp.so kaolin_amd/lib/libkaolin_dibr.so && python tools/bench_rows.py --rows deftet")
done; done
bash tools/gpu_steps.sh "${steps[@]}"

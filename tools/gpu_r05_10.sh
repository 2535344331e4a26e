cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "b8:::200:::python bench.py --no-cpu-baseline --steps 40 > gpurun_out/b8.json" \
 "b1:::200:::python bench.py --no-cpu-baseline --steps 40 --views-per-gpu 1 > gpurun_out/b1.json" \
 "b2:::200:::python bench.py --no-cpu-baseline --steps 40 --views-per-gpu 2 > gpurun_out/b2.json"

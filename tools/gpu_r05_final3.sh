# the C3 bench line against this round's PMC summary, and the 1/2/4-view lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "bench:::300:::python bench.py > gpurun_out/bench_c3.json" \
 "views:::400:::for v in 1 2 4; do python bench.py --no-cpu-baseline --views-per-gpu \$v | grep '^{'; done > gpurun_out/views.jsonl" \
 "lists:::300:::python bench.py --no-cpu-baseline --lists | grep '^{' > gpurun_out/lists.jsonl"

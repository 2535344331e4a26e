# end-of-round evidence, part 1: the GPU suite, the bench lines, timelines, f-row bench rows
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tests:::700:::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:::300:::python bench.py > gpurun_out/bench_c3.json" \
 "views:::400:::for v in 1 2 4; do python bench.py --no-cpu-baseline --views-per-gpu \$v | grep '^{'; done > gpurun_out/views.jsonl" \
 "trace1:::300:::rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr1 -o run -- python3 bench.py --no-cpu-baseline --views-per-gpu 1 --steps 20 > gpurun_out/tr1.out && python3 tools/trace_steps.py gpurun_out/tr1 > gpurun_out/trace_1view.txt" \
 "trace8:::300:::rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8 -o run -- python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/tr8.out && python3 tools/trace_steps.py gpurun_out/tr8 > gpurun_out/trace_8views.txt" \
 "rows:::300:::python tools/bench_rows.py > gpurun_out/bench_rows.jsonl"

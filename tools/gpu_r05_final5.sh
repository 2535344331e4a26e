# end-of-round evidence, part 5: timelines and the f-row bench rows on the final kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "trace1:::300:::rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr1 -o run -- python3 bench.py --no-cpu-baseline --views-per-gpu 1 --steps 20 > gpurun_out/tr1.out && python3 tools/trace_steps.py gpurun_out/tr1 > gpurun_out/trace_1view.txt" \
 "trace8:::300:::rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8 -o run -- python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/tr8.out && python3 tools/trace_steps.py gpurun_out/tr8 > gpurun_out/trace_8views.txt" \
 "rows:::300:::python tools/bench_rows.py > gpurun_out/bench_rows.jsonl"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "prof32:::300:::cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
 "prof64:::300:::cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof64 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype f64 --steps 20 --warmup 5 --no-cpu-baseline" \
 "tr:::60:::python3 tools/trace_steps.py gpurun_out/prof && python3 tools/trace_steps.py gpurun_out/prof64"

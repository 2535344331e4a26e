# the final tree: the GPU suite, smoke() and the default bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "tests:::900:::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:::300:::python bench.py > gpurun_out/bench_final.json"

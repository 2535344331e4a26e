bash tools/gpu_steps.sh \
 "gputests:::900:::python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:::200:::python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:::300:::python3 bench.py"

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "avail:::120:::rocprofv3 --list-avail > gpurun_out/list_avail.txt 2>&1; grep -c . gpurun_out/list_avail.txt" \
 "tnew:::400:::python -u -m pytest tests/test_gpu_step_oracle.py tests/test_gpu_history.py tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread" \
 "tall:::600:::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:::300:::python bench.py --steps 20 --warmup 5" \
 "ab8:::400:::python tools/ab_dirs.py ab/base . 3" \
 "ab1:::400:::python tools/ab_dirs.py ab/base . 3 --views-per-gpu 1" \
 "pert:::600:::python tools/ab_args.py 2 '--perturb 5e-4 --tile-history 1' '--perturb 5e-4 --tile-history 0' && python tools/ab_args.py 2 '--perturb 2e-3 --tile-history 1' '--perturb 2e-3 --tile-history 0' && python bench.py --perturb 2e-3 --no-cpu-baseline > gpurun_out/pert_2e-3.json"

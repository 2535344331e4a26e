cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "prof:::700:::bash tools/profile_c3.sh && bash tools/pmc_mix.sh gpurun_out/pmc --steps 5 --warmup 2 --no-graph && python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt && python3 tools/make_traffic.py gpurun_out/pmc/summary.json gpurun_out/pmc_traffic_c3.json c3 > /dev/null" \
 "flags:::600:::bash tools/pmc_flags.sh 0 1 4 16 32 1024 8192 2>&1 | grep -E 'dibr_fwd|failed'" \
 "pert:::600:::python tools/ab_args.py 2 '--perturb 2e-3 --tile-history 1' '--perturb 2e-3 --tile-history 0' && python tools/ab_args.py 2 '--perturb 1e-2 --tile-history 1' '--perturb 1e-2 --tile-history 0' && python bench.py --perturb 1e-2 --no-cpu-baseline > gpurun_out/pert_1e-2.json"

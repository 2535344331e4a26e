# end-of-round evidence, part 2: kernel-trace stats, the PMC passes (traffic, VALU mix), the configs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "prof:::700:::bash tools/profile_c3.sh && bash tools/pmc_mix.sh gpurun_out/pmc --steps 5 --warmup 2 --no-graph && python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt" \
 "cfgs:::600:::bash tools/bench_configs.sh"

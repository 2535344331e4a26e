cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "dtpmc:::400:::bash tools/pmc_cmd.sh gpurun_out/dtpmc tools/bench_rows.py --rows deftet --dt-fwd --steps 5 && python tools/pmc_summary.py gpurun_out/dtpmc > gpurun_out/dtpmc/summary.txt"

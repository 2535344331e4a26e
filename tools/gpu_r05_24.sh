cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
 "pmc:::500:::bash tools/pmc_cmd.sh gpurun_out/pmc_dt tools/bench_rows.py --rows deftet --dt-fwd --steps 5 && python tools/pmc_summary.py gpurun_out/pmc_dt > gpurun_out/pmc_dt/summary.txt"

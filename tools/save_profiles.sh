#!/bin/bash
# Copy the judged summaries of a GPU profiling call (tools/profile_c3.sh, tools/bench_configs.sh)
# from gpurun_out/ into profiles/<round>/ with a tag.  Usage: tools/save_profiles.sh r02 [tag]
set -e
cd "$(dirname "$0")/.."
r=${1:-r02}; tag=${2:+_$2}
mkdir -p profiles/$r
[ -f gpurun_out/prof/run_kernel_stats.csv ] && cp gpurun_out/prof/run_kernel_stats.csv profiles/$r/rocprof_kernel_stats_c3$tag.csv
[ -f gpurun_out/pmc_summary.txt ] && cp gpurun_out/pmc_summary.txt profiles/$r/pmc_summary_c3$tag.txt
[ -f gpurun_out/pmc/summary.json ] && cp gpurun_out/pmc/summary.json profiles/$r/pmc_summary_c3$tag.json && \
  python3 tools/make_traffic.py profiles/$r/pmc_summary_c3$tag.json profiles/$r/pmc_traffic_c3$tag.json c3 f32 8 > /dev/null
[ -f gpurun_out/cfgs.jsonl ] && cp gpurun_out/cfgs.jsonl profiles/$r/bench_configs$tag.jsonl
ls -la profiles/$r

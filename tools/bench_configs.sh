#!/bin/bash
# Bench lines for the other SURVEY §8(d) configs and variants (1 GPU): one JSON line each into
# gpurun_out/cfgs.jsonl.  Any failing run ends the sequence.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/cfgs.jsonl; : > $out
for a in "--config c2" "--config c2 --dtype f64" "--config c3 --dtype f64" \
         "--config c3 --lists" "--config c3 --views-per-gpu 1" "--config c3 --views-per-gpu 1 --no-graph" \
         "--config c3 --views-per-gpu 2" "--config c3 --views-per-gpu 4" \
         "--config c4 --sigmainv 3000 --boxlen 0.05" "--config c4 --sigmainv 7000 --boxlen 0.02" \
         "--config c4 --sigmainv 17000 --boxlen 0.02" "--config c4 --sigmainv 30000 --boxlen 0.01" \
         "--config c5" "--config c5soup" "--config c3 --iou fused" "--config c3 --iou compose"; do
  echo "== $a"
  timeout -k 10 180 python bench.py --no-cpu-baseline $a | grep '^{' >> $out
  tail -c 300 $out; echo
done

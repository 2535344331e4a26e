#!/bin/bash
# The GPU-box command sets of this repository, by name (replaces the round-5 one-off scripts).
# Usage (on the box, through gpurun): bash tools/gpu_run.sh PRESET [PRESET ...]
# Presets (each one step of tools/gpu_steps.sh, with its own time limit; the first failing step
# ends the call):
#   tests      the whole GPU suite                       quick   the suite without f2/f3/f4 rows
#   smoke      __graft_entry__.smoke()                   bench   the C3 bench line (bench_c3.json)
#   views      1 / 2 / 4-view bench lines (views.jsonl)  lists   the --lists bench line
#   trace1     rocprof kernel trace of the 1-view graph replays (trace_1view.txt)
#   trace8     the same at 8 views (trace_8views.txt)
#   rows       the f-row bench lines (bench_rows.jsonl)  cfgs    the C2-C5 bench lines
#   prof       rocprof stats + the PMC passes of the C3 step (pmc_summary.txt)
#   ab8 / ab1  same-box A/B of ab/base (tools/ab_prepare.sh REV base) against this tree, 8 / 1 views
#   ab2        the same at 2 views
#   spawn      bench.py --gpus 2 starting its own ranks (gloo, sharing the one GPU)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd "$ROOT" || exit 2
T="--timeout 120 --timeout-method thread"
steps=()
for p in "$@"; do
  case "$p" in
    tests) steps+=("tests:::700:::python -u -m pytest tests -m gpu -x -q $T") ;;
    quick) steps+=("quick:::500:::python -u -m pytest tests -m gpu -x -q $T --ignore tests/test_gpu_f2.py --ignore tests/test_gpu_f3.py --ignore tests/test_gpu_f4.py") ;;
    smoke) steps+=("smoke:::200:::python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) steps+=("bench:::300:::python bench.py > gpurun_out/bench_c3.json") ;;
    views) steps+=("views:::400:::for v in 1 2 4; do python bench.py --no-cpu-baseline --views-per-gpu \$v | grep '^{'; done > gpurun_out/views.jsonl") ;;
    lists) steps+=("lists:::300:::python bench.py --no-cpu-baseline --lists | grep '^{' > gpurun_out/lists.jsonl") ;;
    trace1) steps+=("trace1:::300:::rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr1 -o run -- python3 bench.py --no-cpu-baseline --views-per-gpu 1 --steps 20 > gpurun_out/tr1.out && python3 tools/trace_steps.py gpurun_out/tr1 > gpurun_out/trace_1view.txt") ;;
    trace8) steps+=("trace8:::300:::rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8 -o run -- python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/tr8.out && python3 tools/trace_steps.py gpurun_out/tr8 > gpurun_out/trace_8views.txt") ;;
    rows) steps+=("rows:::300:::python tools/bench_rows.py > gpurun_out/bench_rows.jsonl") ;;
    cfgs) steps+=("cfgs:::600:::bash tools/bench_configs.sh") ;;
    prof) steps+=("prof:::700:::bash tools/profile_c3.sh && bash tools/pmc_mix.sh gpurun_out/pmc --steps 5 --warmup 2 --no-graph && python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt") ;;
    ab8) steps+=("ab8:::400:::python tools/ab_dirs.py ab/base . 3") ;;
    ab2) steps+=("ab2:::400:::python tools/ab_dirs.py ab/base . 3 --views-per-gpu 2") ;;
    ab1) steps+=("ab1:::400:::python tools/ab_dirs.py ab/base . 3 --views-per-gpu 1") ;;
    spawn) steps+=("spawn:::200:::KD_BENCH_BACKEND=gloo python bench.py --gpus 2 --views-per-gpu 1 --steps 5 --no-weak > gpurun_out/spawn2.json") ;;
    *) echo "unknown preset: $p" >&2; exit 2 ;;
  esac
done
bash tools/gpu_steps.sh "${steps[@]}"

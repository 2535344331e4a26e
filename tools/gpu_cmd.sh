cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
bash tools/gpu_steps.sh \
 "kaoff:::300:::cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ka0 -o run -- $B" \
 "kaon:::300:::cd /tmp && HIP_FORCE_DEV_KERNARG=1 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ka1 -o run -- $B" \
 "b0:::200:::$B" \
 "b1:::200:::HIP_FORCE_DEV_KERNARG=1 $B" \
 "tr:::60:::python3 tools/trace_steps.py gpurun_out/ka0 && python3 tools/trace_steps.py gpurun_out/ka1"
for f in b0 b1; do python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1])
print('$f', d['ms_per_step'])"; done

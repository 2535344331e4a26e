B="python3 bench.py --dtype f64 --steps 30 --warmup 5 --no-cpu-baseline"
bash tools/gpu_steps.sh \
 "f64base:::200:::cd ab/base && $B" \
 "f64new:::200:::$B" \
 "f64base2:::200:::cd ab/base && $B" \
 "f64new2:::200:::$B" \
 "f32new:::200:::python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline" \
 "gputests:::900:::python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
for f in f64base f64new f64base2 f64new2 f32new; do python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1])
print('$f', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"; done

set -e
cd $GRAFT_REPO_ROOT
out=gpurun_out/cfgs.jsonl; : > $out
for a in "--config c2" "--config c4 --sigmainv 3000 --boxlen 0.05" "--config c4 --sigmainv 7000 --boxlen 0.02" "--config c4 --sigmainv 17000 --boxlen 0.02" "--config c4 --sigmainv 30000 --boxlen 0.01" "--config c5" "--config c5soup"; do
  echo "== $a"
  timeout -k 10 180 python bench.py --no-cpu-baseline $a | grep '^{' >> $out
  tail -c 400 $out
done

# A/B of environment settings on one box: for each "VAR=VAL[,VAR=VAL]" spec (or "base"), the quick
# configs[2] step (bench.py, 10 steps) and rank 0's part of the 8-way split (tools/split_part.py),
# each under its own time limit; stops at the first failure.   bash tools/ab_env.sh TAG SPEC ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  envs=""; [ "$spec" != base ] && envs=$(echo "$spec" | tr ',' ' ')
  f=$(echo "$spec" | tr -c 'A-Za-z0-9_\n' '_')
  env $envs timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/q_$f.json 2> $OUT/q_$f.log || { tail -20 $OUT/q_$f.log; exit 1; }
  env $envs timeout -k 10 120 python -u tools/split_part.py 0 8 7 > $OUT/p_$f.log 2>&1 || { tail -20 $OUT/p_$f.log; exit 1; }
  python -c "
import json, re
d = json.load(open('$OUT/q_$f.json'))
t = sorted(float(x) for x in re.findall(r', ([0-9.]+) ms,', open('$OUT/p_$f.log').read())[2:])
print('%-40s step %.2f ms  part0/8 median %.3f ms min %.3f' % ('$spec', d['ms_per_step'], t[len(t) // 2], t[0]))"
done

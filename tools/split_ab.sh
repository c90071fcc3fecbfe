# Same-box A/B of the multi-GPU row split: the quick configs[2] step plus the serial per-part
# rehearsal (bench.py split_rehearsal) for each "VAR=VAL[,VAR=VAL]" spec (or "base").
#   bash tools/split_ab.sh TAG SPEC ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  envs=""; [ "$spec" != base ] && envs=$(echo "$spec" | tr ',' ' ')
  f=$(echo "$spec" | tr -c 'A-Za-z0-9_\n' '_')
  env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-cfg5 > $OUT/s_$f.json 2> $OUT/s_$f.log || { tail -20 $OUT/s_$f.log; exit 1; }
  python -c "
import json
d = json.load(open('$OUT/s_$f.json'))
s = d['split_rehearsal']
print('%-24s step %.2f ms' % ('$spec', d['ms_per_step']), ' '.join('%s-way eff %.3f max %.3f mean %.3f' % (k, v['projected_efficiency'], max(v['part_ms']), sum(v['part_ms']) / len(v['part_ms'])) for k, v in s.items()))"
done

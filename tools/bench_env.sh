# GPU-box: short headline bench under a list of environment settings, one JSON line each.
#   bash tools/bench_env.sh TAG "GMAT_LR_RANK=384" "GMAT_LR_RANK=512"
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
k=0
for e in "$@"; do
  k=$((k+1))
  env $e timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff > $OUT/bench_$k.json 2> $OUT/bench_$k.log || { tail -20 $OUT/bench_$k.log; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$k.json')); s=d['scan']; r=d['roofline']; print('$e', '%.3g pairs/s' % d['value'], '%.1f ms/step' % d['ms_per_step'], 'cand %d' % s['candidates_per_step'], 'screen %.3f side %.3f refine %.3f' % (s['screen_s_per_step_rank0'], s['side_s_per_step_rank0'], s['refine_s_per_step_rank0']), 'frac %.3f' % r['frac'])"
done

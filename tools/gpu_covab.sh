# GPU-box: same-box interleaved A/B of an environment switch ($1: VAR=VALUE) on the covariate-design
# leg of the bench (configs[2] cohort with three covariates)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${2:-covab}
mkdir -p $OUT
VAR=${1%%=*}
VAL=${1#*=}
for r in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export $VAR=$VAL; else unset $VAR; fi
    timeout -k 10 300 python bench.py --steps 3 --no-cpu --no-grm --no-eff --no-e2e --no-split --no-cfg5 --no-reml > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { tail -20 $OUT/bench_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); c=d['covariates']; print('$v run $r step %.2f ms, covariates %.2f ms, hits %d' % (d['ms_per_step'], c['ms_per_step'], c['hits']))"
  done
done

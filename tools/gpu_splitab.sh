# GPU-box: same-box interleaved A/B of an environment switch ($1: VAR=VALUE) on the bench's split
# rehearsal (each part of the parallel=[N,k] split timed alone)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${2:-splitab}
mkdir -p $OUT
VAR=${1%%=*}
VAL=${1#*=}
for r in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export $VAR=$VAL; else unset $VAR; fi
    timeout -k 10 300 python bench.py --steps 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-cfg5 --no-reml > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { tail -20 $OUT/bench_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); s=d['split_rehearsal']; print('$v run $r step %.2f ms, parts' % d['ms_per_step'], {k: round(x['projected_step_ms'], 2) for k, x in s.items()})"
  done
done

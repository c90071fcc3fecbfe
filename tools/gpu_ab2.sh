# GPU-box: same-box A/B of an environment switch ($1) on the scan-only bench line, interleaved
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab2
mkdir -p $OUT
for r in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then export $1=1; else unset $1; fi
    timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { tail -20 $OUT/bench_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v run $r ms/step %.2f identical %s' % (d['ms_per_step'], d['parity']['full_triangle']['identical']))"
  done
done

# GPU-box: GPU tests (skipped when NOTESTS=1), then a same-box interleaved A/B of an environment
# switch ($1: VAR or VAR=VALUE) on the scan-only bench line (base = VAR unset)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${2:-pfab}
mkdir -p $OUT
if [ -z "$NOTESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
VAR=${1%%=*}
case "$1" in *=*) VAL=${1#*=} ;; *) VAL=1 ;; esac
for r in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then export $VAR=$VAL; else unset $VAR; fi
    timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 --no-reml > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { tail -20 $OUT/bench_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); r=d['roofline']; print('$v run $r ms/step %.2f identical %s pf %.1f us frac %.3f' % (d['ms_per_step'], d['parity']['full_triangle']['identical'], r['avg_launch_ms']*1e3, r['frac']))"
  done
done

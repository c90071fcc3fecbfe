# GPU-box: full GPU tests, REML alone, scan bench with early vs late refine
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python3 tools/reml_only.py > $OUT/reml.out 2>&1 || { tail -20 $OUT/reml.out; exit 1; }
grep REML $OUT/reml.out
for v in early late; do
  if [ $v = late ]; then export GMAT_LATE_REFINE=1; fi
  timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -20 $OUT/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v ms/step %.2f value %.3e identical %s' % (d['ms_per_step'], d['value'], d['parity']['full_triangle']['identical']))"
done

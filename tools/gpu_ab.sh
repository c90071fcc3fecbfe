# GPU-box: GPU tests, then the scan-only bench line three times (box-to-box noise is ~5 %)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { tail -20 $OUT/bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$r.json')); print('run $r ms/step %.2f value %.3e identical %s' % (d['ms_per_step'], d['value'], d['parity']['full_triangle']['identical']))"
done

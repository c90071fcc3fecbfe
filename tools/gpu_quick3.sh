# GPU-box: quick check of a scan change -- full-triangle + cfg3 parity tests, a short bench, rocprof kernel stats
set -o pipefail
export TMPDIR=/tmp
T=${1:-q}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_full_triangle.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-cfg5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('value %.4g ms %.2f dominant %s %.1f us frac %.3f ft %s' % (d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms']*1e3, r['frac'], d['parity']['full_triangle'].get('identical'))); print(json.dumps(r.get('kernels'))); print(d['split_rehearsal']['8'] if d.get('split_rehearsal') else '')"
cd /tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/prof.out 2>&1 || { tail -20 $OUT/prof.out; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-160
if [ -n "$LIVE" ]; then
  GMAT_LIVE_COUNT=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/live.json 2> $OUT/live.err || { tail -5 $OUT/live.err; exit 1; }
  grep "prefilter keeps" $OUT/live.err | tail -3
fi
if [ -n "$STAMPS" ]; then
  GMAT_PF_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/stamps.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
  grep "prefilter launch" $OUT/stamps.err | tail -3
fi

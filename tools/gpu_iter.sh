# GPU-box iteration: the GPU test suite (or the files in $TESTS), then a scan-only bench line
# (parity against the stored full-triangle hit set included) and rocprof kernel stats of 2 steps.
set -o pipefail
export TMPDIR=/tmp
T=${1:-iter}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step %.2f value %.3e' % (d['ms_per_step'], d['value'])); print(json.dumps(d['roofline']['kernels'])); print(d['parity']['full_triangle'])"
cd /tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/prof.out 2>&1 || { tail -20 $OUT/prof.out; exit 1; }
python3 tools/step_timeline.py $OUT/prof/run_kernel_trace.csv

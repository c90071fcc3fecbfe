# GPU-box: the whole GPU test suite, the default bench line, rocprof kernel stats of a short run
set -o pipefail
export TMPDIR=/tmp
T=${1:-full}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/trace_gaps.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) lr_screen_kernel 98

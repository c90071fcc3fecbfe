# GPU-box: GPU test suite, default bench line, rocprof kernel stats, PMC passes of the two scan kernels
set -o pipefail
export TMPDIR=/tmp
T=${1:-r3c}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/prof.out 2>&1 || { tail -20 $OUT/prof.out; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec head -14 {} \;
KEY="lrc_screen_kernel|prefilter_pass_kernel" bash tools/pmc.sh ${T}_pmc || exit 1
for k in lrc_screen_kernel prefilter_pass_kernel; do
  python3 tools/pmc_summary.py gpurun_out/${T}_pmc $k --out gpurun_out/${T}_pmc/traffic_$k.json --level -1 --rank 128 --n-id 2000 --n-snp 50000 || exit 1
done

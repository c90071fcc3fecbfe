# GPU-box: configs[1] REML alone (tools/reml_only.py) under rocprof kernel stats + trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-remlprof}
mkdir -p $OUT
cd /tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/reml_only.py > $OUT/reml.out 2>&1 || { tail -20 $OUT/reml.out; exit 1; }
grep REML $OUT/reml.out
head -14 $OUT/prof/run_kernel_stats.csv | cut -c1-160

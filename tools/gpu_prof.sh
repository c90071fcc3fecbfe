# GPU-box: rocprofv3 kernel trace + stats of a short headline run ($2: env settings), gap analysis
set -o pipefail
export TMPDIR=/tmp
T=${1:-prof}
OUT=gpurun_out/$T
mkdir -p $OUT
env ${2:-GMAT_X=0} timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/trace_gaps.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) lr_screen_kernel 98
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {} | cut -c1-150'

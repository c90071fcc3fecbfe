# GPU-box: rocprofv3 kernel stats of the effect-screen bench (eff_screen_kernel / eff_exact_kernel)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-effprof}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-cov --no-e2e --cpu-budget 0.5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep -i "eff" $(find $OUT/prof -name "*kernel_stats.csv" | head -1) | cut -c1-200

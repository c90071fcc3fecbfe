set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$1/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml --covariates > gpurun_out/$1/prof.log 2>&1 || { tail -20 gpurun_out/$1/prof.log; exit 1; }
find gpurun_out/$1/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {} | cut -c1-220'
grep -v "^$" gpurun_out/$1/prof.log | grep '"value"' | cut -c1-300

#!/bin/bash
# GPU-box routine: parity tests, then a short bench, then a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; the script stops at the first failure.
#   bash tools/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-run}
KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then KARG=(-k "$KEXPR"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
if [ "${BENCH:-1}" = "1" ]; then
  GMAT_DEBUG=1 timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-budget 10 > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
  cat $OUT/bench.json
fi
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -14 {} | cut -c1-180'
fi

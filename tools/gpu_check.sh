#!/bin/bash
# GPU-box routine: parity tests, then a short bench, then a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-budget 10 > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-grm > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {}'
fi

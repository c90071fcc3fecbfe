# GPU-box quick check: parity tests (-k filter optional), then a short headline bench.
set -o pipefail
TAG=${1:-q}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then KARG="-k $K"; else KARG=""; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider $KARG > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
GMAT_DEBUG=${GMAT_DEBUG:-} timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.json

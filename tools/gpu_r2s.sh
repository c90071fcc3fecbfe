# GPU-box: parity subset, then the headline step under tile-per-workgroup settings, then stamps
set -o pipefail
export TMPDIR=/tmp
T=${1:-r2s}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "${KEXPR:-tiny or mouse or cfg3 or covariates or threshold or plan_state}" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/bench_env.sh $T ${ENVS:-GMAT_LR_TPW=1 GMAT_LR_TPW=2 GMAT_LR_TPW=4 GMAT_LR_TPW=8 GMAT_LR_TPW=13} || exit 1
GMAT_LR_STAMPS=1 GMAT_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml > $OUT/stamps.json 2> $OUT/stamps.log || { tail -20 $OUT/stamps.log; exit 1; }
grep "lr stamps" $OUT/stamps.log

# GPU-box: parity subset, headline bench, PMC passes 1-2 of the low-rank screen
set -o pipefail
export TMPDIR=/tmp
T=${1:-r2x}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "${KEXPR:-tiny or cfg3}" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/bench_env.sh $T ${ENVS:-GMAT_X=0} || exit 1
PASSES="${PASSES:-1 2}" NSNP=50000 KEY=${KEY:-lr_screen} ARGS="bench.py --steps 1 --warmup 0 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml" bash tools/pmc.sh ${T}_pmc || exit 1
python3 tools/pmc_summary.py gpurun_out/${T}_pmc ${KEY:-lr_screen}

# GPU-box: parity subset (incl. the int8 levels: lazily computed bounds), headline bench, PMC passes
# of the low-rank screen (heartbeat on stdout while the counter passes run)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r2v}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "tiny or mouse or cfg3 or covariates or threshold or plan_state or vs_oracle" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/bench_env.sh $T GMAT_X=0 || exit 1
( while sleep 50; do echo "pmc running $(date +%T)"; done ) &
HB=$!
NSNP=${NSNP:-10000} KEY=${KEY:-lr_screen} ARGS="bench.py --n-snp ${NSNP:-10000} --steps 1 --warmup 0 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml" bash tools/pmc.sh ${T}_pmc
rc=$?
kill $HB
[ $rc -eq 0 ] || exit 1
python3 tools/pmc_summary.py gpurun_out/${T}_pmc ${KEY:-lr_screen}

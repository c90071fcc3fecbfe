# GPU-box: parity subset, low-rank screen timing diagnostics, stamps, the default bench line, rocprof summary
set -o pipefail
export TMPDIR=/tmp
T=${1:-r2r}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "${KEXPR:-tiny}" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/lr_diag.py --modes 0,1,2,3 --rounds 2 > $OUT/diag.log 2>&1 || { tail -20 $OUT/diag.log; exit 1; }
grep diag $OUT/diag.log
GMAT_LR_STAMPS=1 GMAT_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml > $OUT/stamps.json 2> $OUT/stamps.log || { tail -20 $OUT/stamps.log; exit 1; }
grep "lr stamps" $OUT/stamps.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -14 {} | cut -c1-180'

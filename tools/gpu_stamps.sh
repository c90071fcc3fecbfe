# GPU-box: per-workgroup phase stamps of the low-rank screen for GMAT_LR_DIAG modes ($2)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-stamps}
mkdir -p $OUT
for d in ${2:-0}; do
  GMAT_LR_DIAG=$d GMAT_LR_STAMPS=1 GMAT_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml > $OUT/stamps_$d.json 2> $OUT/stamps_$d.log || { tail -20 $OUT/stamps_$d.log; exit 1; }
  echo "== diag $d"; grep "lr stamps" $OUT/stamps_$d.log | head -6
done

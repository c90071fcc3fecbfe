# GPU-box: low-rank screen timing diagnostics only (GMAT_LR_DIAG modes given as $2)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
timeout -k 10 400 python -u tools/lr_diag.py --modes ${2:-0,1,2,3,4,7,8} --rounds 2 > $OUT/diag.log 2>&1 || { tail -20 $OUT/diag.log; exit 1; }
grep diag $OUT/diag.log

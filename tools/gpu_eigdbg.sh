set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/eigdbg
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_gpu_eig.py -q --timeout 100 -p no:cacheprovider > $OUT/split.log 2>&1; echo "split rc $?"; tail -3 $OUT/split.log
GMAT_DGEMM_NOSPLIT=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_eig.py -q --timeout 100 -p no:cacheprovider > $OUT/nosplit.log 2>&1; echo "nosplit rc $?"; tail -3 $OUT/nosplit.log
GMAT_DEBUG=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_eig.py -q -s --timeout 100 -p no:cacheprovider > $OUT/dbg.log 2>&1; echo "debug rc $?"; grep -c sym_eig $OUT/dbg.log; tail -3 $OUT/dbg.log
exit 0

# GPU-box: the eigensolver tests, then GMAT_DEBUG plan setup timing at configs[2]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/eig
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_eig.log 2>&1 || { tail -40 $OUT/pytest_eig.log; exit 1; }
tail -8 $OUT/pytest_eig.log

# GPU-box: full-triangle audit -- the small-cohort GPU test, then configs[2] AA over all 1.25e9 pairs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_triangle.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -5 $OUT/pytest.log
timeout -k 10 900 python -u tools/full_triangle.py --out $OUT > $OUT/full_triangle.log 2>&1 || { tail -30 $OUT/full_triangle.log; exit 1; }
tail -12 $OUT/full_triangle.log

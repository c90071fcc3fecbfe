# GPU-box: full GPU tests, REML alone with and without the captured Cholesky graph
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/remlg
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python3 tools/reml_only.py > $OUT/reml_graph.out 2>&1 || { tail -20 $OUT/reml_graph.out; exit 1; }
grep REML $OUT/reml_graph.out
GMAT_REML_NO_GRAPH=1 timeout -k 10 120 python3 tools/reml_only.py > $OUT/reml_direct.out 2>&1 || { tail -20 $OUT/reml_direct.out; exit 1; }
grep REML $OUT/reml_direct.out

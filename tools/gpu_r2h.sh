set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2h
timeout -k 10 600 python -u -m pytest tests/test_gpu_cfg5.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2h/pytest.log 2>&1 || { tail -40 gpurun_out/r2h/pytest.log; exit 1; }
tail -6 gpurun_out/r2h/pytest.log
GMAT_DEBUG=1 timeout -k 10 600 python bench.py --config cfg5 > gpurun_out/r2h/cfg5.json 2> gpurun_out/r2h/cfg5.log || { tail -20 gpurun_out/r2h/cfg5.log; exit 1; }
cat gpurun_out/r2h/cfg5.json

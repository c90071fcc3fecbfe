# GPU-box: full GPU test suite, then tools/gpu_final.sh (bench line, rocprof, PMC)
set -o pipefail
export TMPDIR=/tmp
T=${1:-final}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
bash tools/gpu_final.sh $T

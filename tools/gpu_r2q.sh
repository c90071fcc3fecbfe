# GPU-box: full check at HEAD (tests, bench, rocprof) plus the low-rank screen's per-workgroup stamps
set -o pipefail
export TMPDIR=/tmp
BENCH=1 PROF=1 bash tools/gpu_check.sh ${1:-r2q} || exit 1
GMAT_LR_STAMPS=1 GMAT_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml > gpurun_out/${1:-r2q}/stamps.json 2> gpurun_out/${1:-r2q}/stamps.log || exit 1
grep "lr stamps" gpurun_out/${1:-r2q}/stamps.log | head -8

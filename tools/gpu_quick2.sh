# GPU-box: correctness subset, then a short headline bench (one JSON summary line)
set -o pipefail
export TMPDIR=/tmp
T=${1:-q}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${2:-mouse or tiny or large_n or vs_oracle_rows or deterministic or cfg3_strat or covariates}" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
if [ $# -ge 2 ]; then shift 2; else shift $#; fi
bash tools/bench_env.sh $T "GMAT_X=0" "$@"

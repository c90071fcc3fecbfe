set -o pipefail
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "mouse or tiny or large_n or vs_oracle_rows or deterministic" > gpurun_out/r2e/pytest.log 2>&1 || { tail -30 gpurun_out/r2e/pytest.log; exit 1; }
tail -2 gpurun_out/r2e/pytest.log
bash tools/bench_env.sh r2e "GMAT_LR_WAVES=8" "GMAT_LR_WAVES=4" || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-reml > gpurun_out/r2e/cov.json 2> gpurun_out/r2e/cov.log || { tail gpurun_out/r2e/cov.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2e/cov.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['covariates']))"

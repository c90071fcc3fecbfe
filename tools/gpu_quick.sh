set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/s1/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s1/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s1/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.log || { tail -20 gpurun_out/s1/bench.log; exit 1; }
cat gpurun_out/s1/bench.json

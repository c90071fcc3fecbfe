# GPU-box: full GPU tests, scan bench, prefilter stamps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step %.2f value %.3e pf %.3f ms/launch identical %s' % (d['ms_per_step'], d['value'], d['roofline']['kernels']['prefilter_pass_kernel']['avg_launch_ms'], d['parity']['full_triangle']['identical']))"
bash tools/gpu_pfstamps.sh ${1:-r3e}_stamps

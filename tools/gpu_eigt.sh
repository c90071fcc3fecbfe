# GPU-box: full GPU tests, then plan-setup timing with the eigensolver's debug breakdown (configs[2])
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/eigt
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
GMAT_DEBUG=1 timeout -k 10 200 python bench.py --steps 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep -E "sym_eig_bottom.*iterations|lr_setup|prefilter mu" $OUT/bench.err | head -12
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step %.2f' % d['ms_per_step']); print(d['setup']); print(d['parity']['full_triangle']['identical'])"

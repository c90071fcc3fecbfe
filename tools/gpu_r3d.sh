# GPU-box: full GPU tests, scan bench (two-stream prefilter vs one), eig debug line, prefilter stamps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for v in two one; do
  if [ $v = one ]; then export GMAT_PF_ONE_STREAM=1; fi
  timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -20 $OUT/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v ms/step %.2f value %.3e pf %.3f ms/launch identical %s' % (d['ms_per_step'], d['value'], d['roofline']['kernels']['prefilter_pass_kernel']['avg_launch_ms'], d['parity']['full_triangle']['identical'])); print(d['setup'])"
done
unset GMAT_PF_ONE_STREAM
GMAT_DEBUG=1 timeout -k 10 100 python bench.py --steps 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/dbg.json 2> $OUT/dbg.err || { tail -20 $OUT/dbg.err; exit 1; }
grep -E "sym_eig_bottom.*iterations|lr_setup" $OUT/dbg.err | head -3
bash tools/gpu_pfstamps.sh r3d_stamps

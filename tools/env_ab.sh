# configs[2] step (bench.py, full-triangle parity on) under several environment settings, in turn,
# twice each in alternating order: bash tools/env_ab.sh OUT 'name=ENV=val,ENV2=val' 'name2=' ...
# (BENCH_EXTRA=--covariates: the covariate design's step; its parity is the GPU tests')
out=gpurun_out/$1; shift
mkdir -p $out
for rep in 1 2; do
  for arm in "$@"; do
    name=${arm%%=*}; envs=${arm#*=}
    env_args=$(echo "$envs" | tr ',' ' ')
    env $env_args timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 $BENCH_EXTRA > $out/$name.$rep.json 2> $out/$name.$rep.log || { echo "arm $name failed"; tail -5 $out/$name.$rep.log; exit 1; }
    python3 -c "import json; d=json.load(open('$out/$name.$rep.json')); k=d.get('roofline', {}).get('kernels', {}).get('prefilter_pass_kernel', {}); print('%-10s rep $rep: %.2f ms per step, prefilter %.3f ms per launch, %d candidates, parity %s' % ('$name', d['ms_per_step'], k.get('avg_launch_ms', 0.0), d.get('scan', {}).get('candidates_per_step', -1), d.get('parity', {}).get('full_triangle', {}).get('identical')))"
  done
done

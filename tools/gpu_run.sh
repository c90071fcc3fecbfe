# GPU-box driver for this round's checks: stages given as arguments, each under its own time limit,
# stopping at the first failure.  Output under gpurun_out/<tag>/.
#   bash tools/gpu_run.sh TAG tests|bench|bench_cfg5|prof ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for st in "$@"; do
  case $st in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
      tail -3 $OUT/tests.log ;;
    scantests)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_pair_screen.py tests/test_gpu_lr_variants.py tests/test_gpu_parity.py tests/test_gpu_full_triangle.py -x -q --timeout 240 --timeout-method thread > $OUT/scantests.log 2>&1 || { tail -40 $OUT/scantests.log; exit 1; }
      tail -2 $OUT/scantests.log ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log || { tail -30 $OUT/bench.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/bench.json')); print('value %.4g ms %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))" ;;
    quick)
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/quick.json 2> $OUT/quick.log || { tail -30 $OUT/quick.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/quick.json')); print('value %.4g ms %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))" ;;
    cfg5|cfg5f0|cfg5f2|cfg5f10)
      FS=5; case $st in cfg5f0) FS=0;; cfg5f2) FS=2;; cfg5f10) FS=10;; esac
      timeout -k 10 600 python -u bench.py --config cfg5 --family-size $FS --cfg5-reps ${CFG5_REPS:-3} > $OUT/$st.json 2> $OUT/$st.log || { tail -30 $OUT/$st.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$st.json')); r=d['reml']; print('$st', 'value %.3g' % d['value'], 'iters', r['iters'], 'var', [round(v, 4) for v in r['var']], 'grad', r.get('grad_norm_last5'), 'upd', r.get('update_norm_last5'), 'emw', r.get('em_weight_last5'), 'DD cand', d['epiDD']['candidates'], 'AD cand', d['epiAD']['candidates'], 'DD s', d['epiDD']['s'])" ;;
    prof|serial)
      # kernel trace + stats of a short scan run and the step timeline of its last step; serial: the
      # same with kernels serialised (AMD_SERIALIZE_KERNEL=3), so the per-kernel sums are standalone times
      SER=""; [ $st = serial ] && SER="AMD_SERIALIZE_KERNEL=3"
      env $SER timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$st -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/${st}_bench.json 2> $OUT/$st.log || { tail -30 $OUT/$st.log; exit 1; }
      python3 tools/step_timeline.py $(find $OUT/$st -name "*kernel_trace.csv" | head -1) | tee $OUT/${st}_timeline.txt ;;
    *)
      echo "unknown stage $st"; exit 2 ;;
  esac
done

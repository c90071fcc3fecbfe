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
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log || { tail -30 $OUT/bench.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/bench.json')); print('value %.4g ms %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))" ;;
    quick)
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/quick.json 2> $OUT/quick.log || { tail -30 $OUT/quick.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/quick.json')); print('value %.4g ms %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))" ;;
    cfg5)
      timeout -k 10 600 python -u bench.py --config cfg5 > $OUT/cfg5.json 2> $OUT/cfg5.log || { tail -30 $OUT/cfg5.log; exit 1; }
      tail -c 1500 $OUT/cfg5.json ;;
    prof)
      cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $GRAFT_REPO_ROOT/$OUT/prof_bench.json 2> $GRAFT_REPO_ROOT/$OUT/prof.log || { tail -30 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
      cd $GRAFT_REPO_ROOT ;;
    *)
      echo "unknown stage $st"; exit 2 ;;
  esac
done

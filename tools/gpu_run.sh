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
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
      tail -3 $OUT/tests.log ;;
    newtests)
      # this round's limit / buffer / launch tests
      timeout -k 10 1100 python -u -m pytest tests/test_gpu_buffers.py tests/test_gpu_limits.py tests/test_launch.py -m gpu -v --timeout 600 --timeout-method thread > $OUT/newtests.log 2>&1 || { tail -60 $OUT/newtests.log; exit 1; }
      tail -3 $OUT/newtests.log ;;
    serial)
      # every kernel's standalone time (launches serialised), summed over 5 timed configs[2] steps
      AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/serial.json 2> $OUT/serial.log || { tail -20 $OUT/serial.log; exit 1; }
      cp $(find $OUT/serial -name "*kernel_stats.csv" | head -1) $OUT/serial_kernel_stats.csv
      head -12 $OUT/serial_kernel_stats.csv | cut -c1-200 ;;
    timeline)
      # the overlapped step: kernel trace of 5 timed configs[2] steps, the last step's window
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tl -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/tl.json 2> $OUT/tl.log || { tail -20 $OUT/tl.log; exit 1; }
      cp $(find $OUT/tl -name "*kernel_stats.csv" | head -1) $OUT/tl_kernel_stats.csv
      python3 tools/step_timeline.py $(find $OUT/tl -name "*kernel_trace.csv" | head -1) > $OUT/step_timeline.txt
      head -30 $OUT/step_timeline.txt ;;
    reml)
      # configs[1] REML under a kernel trace: per-kernel totals of the REML legs (tools/reml_only.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/reml -o run -- python3 tools/reml_only.py 2000 20000 > $OUT/reml.json 2> $OUT/reml.log || { tail -20 $OUT/reml.log; exit 1; }
      cp $(find $OUT/reml -name "*kernel_stats.csv" | head -1) $OUT/reml_kernel_stats.csv
      cat $OUT/reml.json; head -12 $OUT/reml_kernel_stats.csv | cut -c1-160 ;;
    cfg5probe)
      # configs[4] REML convergence on full-sib cohorts (tools/cfg5_reml_probe.py), family sizes 5, 10, 20
      for f in 5 10 20; do
        timeout -k 10 240 python3 -u tools/cfg5_reml_probe.py $f 200 "0.3,0.1,0.1,0.05,0.05,0.4" "0.3,0.1,0.1,0.1,0.1,0.3" > $OUT/cfg5probe_$f.log 2>&1 || { tail -20 $OUT/cfg5probe_$f.log; exit 1; }
        cat $OUT/cfg5probe_$f.log | cut -c1-400
      done ;;
    scantests)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_pair_screen.py tests/test_gpu_lr_variants.py tests/test_gpu_parity.py tests/test_gpu_full_triangle.py -x -q --timeout 240 --timeout-method thread > $OUT/scantests.log 2>&1 || { tail -40 $OUT/scantests.log; exit 1; }
      tail -2 $OUT/scantests.log ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.log || { tail -30 $OUT/bench.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/bench.json')); print('value %.4g ms %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))" ;;
    benchprof)
      # rocprofv3 kernel trace + stats of the driver's default bench command (the roofline's launch times
      # must agree with the stats of the same command)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bp -o run -- python3 bench.py > $OUT/benchprof.json 2> $OUT/benchprof.log || { tail -30 $OUT/benchprof.log; exit 1; }
      cp $(find $OUT/bp -name "*kernel_stats.csv" | head -1) $OUT/bench_kernel_stats.csv
      python3 tools/bench_trace_summary.py $(find $OUT/bp -name "*kernel_trace.csv" | head -1) $OUT/benchprof.json > $OUT/bench_rocprof_summary.txt || exit 1
      cat $OUT/bench_rocprof_summary.txt
      rm -rf $OUT/bp
      head -8 $OUT/bench_kernel_stats.csv | cut -c1-160 ;;
    quick)
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/quick.json 2> $OUT/quick.log || { tail -30 $OUT/quick.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/quick.json')); print('value %.4g ms %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))" ;;
    hostt)
      # host-side phases of each scan (GMAT_HOST_T) and the Python time around the calls
      GMAT_HOST_T=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/hostt.json 2> $OUT/hostt.log || { tail -30 $OUT/hostt.log; exit 1; }
      grep "scan host" $OUT/hostt.log | tail -4 ;;
    stamps)
      # per-tile phase times of one prefilter launch (GMAT_PF_STAMPS: one workgroup per tile, first tile)
      GMAT_PF_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/stamps.json 2> $OUT/stamps.log || { tail -30 $OUT/stamps.log; exit 1; }
      grep "prefilter launch" $OUT/stamps.log | tail -2
      # the same launch with every kernel serialised (no co-running screens): clock and phases alone
      AMD_SERIALIZE_KERNEL=3 GMAT_PF_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/stamps_serial.json 2> $OUT/stamps_serial.log || { tail -30 $OUT/stamps_serial.log; exit 1; }
      grep "prefilter launch" $OUT/stamps_serial.log | tail -1 ;;
    covstamps)
      # per-tile phase times of one covariate prefilter launch (GMAT_PF_STAMPS, one workgroup per tile)
      GMAT_PF_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --covariates --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/covstamps.json 2> $OUT/covstamps.log || { tail -30 $OUT/covstamps.log; exit 1; }
      grep "prefilter launch" $OUT/covstamps.log | tail -1 ;;
    pmc)
      # counter passes of the six scan kernels (one rocprofv3 run per counter group) and their traffic
      # records keyed by the epi stage files' sha256 (bench.py attaches them to roofline.kernels)
      K="prefilter_pass_kernel|lrc_screen_kernel|pair_side_kernel|pair_mxr_kernel|refine8_kernel|refine8_side_kernel"
      KEY="$K" bash tools/pmc.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
      for k in prefilter_pass_kernel lrc_screen_kernel pair_side_kernel pair_mxr_kernel refine8_kernel refine8_side_kernel; do
        python3 tools/pmc_summary.py $OUT/pmc $k --out $OUT/traffic_$k.json --level -1 --rank 128 --n-id 2000 --n-snp 50000 > $OUT/pmc_$k.txt || exit 1
        tail -12 $OUT/pmc_$k.txt
      done ;;
    part)
      # one rank's part of the 8-way split (rank 0), traced: the timeline of a multi-GPU step
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/part -o run -- python3 tools/split_part.py 0 8 5 > $OUT/part.log 2>&1 || { tail -30 $OUT/part.log; exit 1; }
      grep "part 0" $OUT/part.log | tail -3
      python3 tools/step_timeline.py $(find $OUT/part -name "*kernel_trace.csv" | head -1) | tee $OUT/part_timeline.txt
      python3 tools/step_gantt.py $(find $OUT/part -name "*kernel_trace.csv" | head -1) > $OUT/part_gantt.txt
      rm -rf $OUT/part ;;
    parthost)
      # host API trace of rank 0's part (which HIP calls sit between the steps' kernels)
      timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d $OUT/parthost -o run -- python3 tools/split_part.py 0 8 5 > $OUT/parthost.log 2>&1 || { tail -30 $OUT/parthost.log; exit 1; }
      grep "part 0" $OUT/parthost.log | tail -2; ls $OUT/parthost/*/ 2>/dev/null | head; find $OUT/parthost -name "*.csv" | head ;;
    cov)
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --covariates --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/cov.json 2> $OUT/cov.log || { tail -30 $OUT/cov.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/cov.json')); print('covariates: value %.4g ms %.2f' % (d['value'], d['ms_per_step']))" ;;
    covtests)
      timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_workflow.py -x -q --timeout 300 --timeout-method thread > $OUT/covtests.log 2>&1 || { tail -40 $OUT/covtests.log; exit 1; }
      tail -2 $OUT/covtests.log ;;
    cfg5split)
      timeout -k 10 600 python -u bench.py --config cfg5 --cfg5-reps 1 > $OUT/cfg5split.json 2> $OUT/cfg5split.log || { tail -30 $OUT/cfg5split.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/cfg5split.json')); print('cfg5 value %.3g' % d['value'], {k: {n: (round(v['projected_efficiency'], 3), v['hits_match_step']) for n, v in r.items()} for k, r in d['split_rehearsal'].items()})" ;;
    cfg5|cfg5f0|cfg5f2|cfg5f10)
      FS=5; case $st in cfg5f0) FS=0;; cfg5f2) FS=2;; cfg5f10) FS=10;; esac
      timeout -k 10 600 python -u bench.py --config cfg5 --family-size $FS --cfg5-reps ${CFG5_REPS:-3} > $OUT/$st.json 2> $OUT/$st.log || { tail -30 $OUT/$st.log; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$st.json')); r=d['reml']; print('$st', 'value %.3g' % d['value'], 'iters', r['iters'], 'var', [round(v, 4) for v in r['var']], 'grad', r.get('grad_norm_last5'), 'upd', r.get('update_norm_last5'), 'emw', r.get('em_weight_last5'), 'DD cand', d['epiDD']['candidates'], 'AD cand', d['epiAD']['candidates'], 'DD s', d['epiDD']['s'])" ;;
    covprof)
      # kernel trace of the covariate step (prefilter_cov_kernel) and its timeline
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/covprof -o run -- python3 bench.py --steps 3 --warmup 1 --covariates --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/covprof_bench.json 2> $OUT/covprof.log || { tail -30 $OUT/covprof.log; exit 1; }
      python3 tools/step_timeline.py $(find $OUT/covprof -name "*kernel_trace.csv" | head -1) | tee $OUT/covprof_timeline.txt ;;
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

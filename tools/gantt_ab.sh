set -o pipefail
export TMPDIR=/tmp
for arm in ${ARMS:-base p1}; do
  OUT=gpurun_out/r6d/$arm
  mkdir -p $OUT
  GMAT_HIP_LIB=ab/lib_$arm.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/tl.json 2> $OUT/tl.log || { tail -20 $OUT/tl.log; exit 1; }
  python3 tools/step_gantt.py $(find $OUT/tl -name "*kernel_trace.csv" | head -1) > $OUT/gantt.txt || exit 1
  tail -1 $OUT/gantt.txt
  rm -rf $OUT/tl
done

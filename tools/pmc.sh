#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) on the bench's own
# configuration (configs[2] by default: 2,000 x 50,000, one timed step).  Raw output goes to
# gpurun_out/TAG/raw while a pass runs (visible progress) and is deleted after the rows of kernels
# matching the regex $KEY are kept.  PASSES="3 4 5" runs only those passes.
TAG=${1:-pmc}
KEY=${KEY:-"lr_screen_kernel|prefilter_pass_kernel"}
OUT=gpurun_out/$TAG
RAW=gpurun_out/$TAG/raw  # inside gpurun_out so a long pass shows progress; deleted after filtering
mkdir -p $OUT $RAW
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS=${ARGS:-"bench.py --steps 1 --warmup 0 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5"}
i=0
PASSES=${PASSES:-all}
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  if [ "$PASSES" != "all" ] && ! echo " $PASSES " | grep -q " $i "; then continue; fi
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KEY}" --output-format csv -d $RAW/p$i -o run -- python3 $ARGS > $OUT/p$i.out 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.out; exit 1; }
  mkdir -p $OUT/p$i
  for f in run_counter_collection.csv run_kernel_trace.csv; do
    src=$(find $RAW/p$i -name $f | head -1)
    [ -n "$src" ] && { head -1 $src; grep -E "$KEY" $src || true; } > $OUT/p$i/$f
  done
  rm -rf $RAW/p$i
done
rm -rf $RAW
echo done

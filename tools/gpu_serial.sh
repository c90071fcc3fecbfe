# GPU-box: kernel durations with launches serialized (AMD_SERIALIZE_KERNEL=3): each kernel's
# standalone time, summed per kernel over the last timed step
set -o pipefail
export TMPDIR=/tmp
T=${1:-serial}
OUT=gpurun_out/$T
mkdir -p $OUT
AMD_SERIALIZE_KERNEL=3 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-reml > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/trace_gaps.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) lr_screen_kernel 98

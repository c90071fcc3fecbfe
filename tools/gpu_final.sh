# GPU-box: the default bench line (every leg), rocprof kernel stats + trace of a short scan run, and
# the PMC passes of the two scan kernels with their traffic records (keyed by epi.hip's sha256)
set -o pipefail
export TMPDIR=/tmp
T=${1:-final}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('ms/step %.2f value %.3e frac %.3f' % (d['ms_per_step'], d['value'], d['roofline']['frac'])); print('setup', d['setup']); print('reml', d['reml']); print('e2e', d['end_to_end']); print('cfg5', {k: d['cfg5'][k] for k in ('pairs_per_s', 'plan_create_s')}, d['cfg5']['reml'])"
cd /tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/prof.out 2>&1 || { tail -20 $OUT/prof.out; exit 1; }
python3 tools/step_timeline.py $OUT/prof/run_kernel_trace.csv
KEY="lrc_screen_kernel|prefilter_pass_kernel" bash tools/pmc.sh ${T}_pmc || exit 1
for k in lrc_screen_kernel prefilter_pass_kernel; do
  python3 tools/pmc_summary.py gpurun_out/${T}_pmc $k --out gpurun_out/${T}_pmc/traffic_$k.json --level -1 --rank 128 --n-id 2000 --n-snp 50000 > gpurun_out/${T}_pmc/summary_$k.txt || exit 1
  tail -14 gpurun_out/${T}_pmc/summary_$k.txt
done

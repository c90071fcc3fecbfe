# GPU-box: rocprofv3 kernel stats and PMC passes of the GRM (configs[1] agmat, 2,000 x 20,000)
set -o pipefail
TAG=${1:-grm}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GA="tools/grm_only.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GA > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {} | cut -c1-160'
ARGS="$GA" KEY=grm_partial PASSES="${PASSES:-1 2}" bash tools/pmc.sh $TAG/pmc > /dev/null && python3 tools/pmc_summary.py $OUT/pmc grm_partial

# GPU-box: prefilter per-tile phase stamps (launch 5 of a configs[2] step) and the live-pair count
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pfstamps}
mkdir -p $OUT
GMAT_PF_STAMPS=1 GMAT_DEBUG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/stamps.json 2> $OUT/stamps.log || { tail -20 $OUT/stamps.log; exit 1; }
grep -E "prefilter launch" $OUT/stamps.log | head -4

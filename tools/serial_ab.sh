# Serialised kernel times (AMD_SERIALIZE_KERNEL=3, rocprofv3 stats) of the configs[2] step for each
# library arm: bash tools/serial_ab.sh TAG name=lib.so ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for arm in "$@"; do
  name=${arm%%=*}; lib=${arm#*=}
  GMAT_HIP_LIB=$lib AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > $OUT/$name.json 2> $OUT/$name.log || { tail -20 $OUT/$name.log; exit 1; }
  cp $(find $OUT/$name -name "*kernel_stats.csv" | head -1) $OUT/${name}_stats.csv
  rm -rf $OUT/$name
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/${name}_stats.csv')):
    n = r['Name']
    if any(k in n for k in ('prefilter_pass', 'lrc_screen', 'pair_mxr', 'pair_side', 'refine8_kernel', 'lc_fill')):
        print('%-8s %-40s %5s %9.1f us' % ('$name', n.split('(')[0][-40:], r['Calls'], float(r['AverageNs']) / 1e3))"
done

# serialised average launch time of the scan kernels and the overlapped step (configs[2])
mkdir -p gpurun_out/$1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$1/ser -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > gpurun_out/$1/ser.json 2> gpurun_out/$1/ser.log || exit 1
python3 - gpurun_out/$1/ser/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("prefilter_pass", "lrc_screen", "pair_side", "pair_mxr", "lc_fill", "lc_count", "refine8")):
        print("%-40s %5s calls %9.1f us avg" % (n.split("(")[0].replace("void gmat::epi::", "")[:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > gpurun_out/$1/q.json 2> gpurun_out/$1/q.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/$1/q.json')); print('step %.2f ms' % d['ms_per_step'])"
timeout -k 10 200 python3 tools/split_part.py 0 8 6 > gpurun_out/$1/p8.log 2>&1 || exit 1
echo "8-way part 0: $(grep 'part 0' gpurun_out/$1/p8.log | tail -4 | awk '{print $7}' | tr '\n' ' ')"

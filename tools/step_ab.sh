# configs[2] step at several rows-per-launch settings, then rank 0's 4-way part at two
mkdir -p gpurun_out/$1
for rl in ${RLS:-4096 3072 2560}; do
  GMAT_LRC_ROWS=$rl timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-grm --no-eff --no-e2e --no-cov --no-split --no-cfg5 > gpurun_out/$1/s$rl.json 2> gpurun_out/$1/s$rl.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$1/s$rl.json')); print('step rows/launch $rl: %.2f ms' % d['ms_per_step'])"
done
for rl in 2048 3072; do
  GMAT_LRC_ROWS=$rl timeout -k 10 200 python3 tools/split_part.py 0 4 6 > gpurun_out/$1/p4_$rl.log 2>&1 || exit 1
  echo "4-way part rows/launch $rl: $(grep 'part 0' gpurun_out/$1/p4_$rl.log | tail -4 | awk '{print $7}' | tr '\n' ' ')"
done

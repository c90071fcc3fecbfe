# rank 0's 8-way part at several rows-per-launch settings (GMAT_LRC_ROWS), a few reps each
mkdir -p gpurun_out/$1
for rl in ${RLS:-512 768 1024 1536 2048}; do
  GMAT_LRC_ROWS=$rl timeout -k 10 200 python3 tools/split_part.py 0 8 6 > gpurun_out/$1/rl$rl.log 2>&1 || exit 1
  echo "rows/launch $rl: $(grep 'part 0' gpurun_out/$1/rl$rl.log | tail -4 | awk '{print $6}' | tr '\n' ' ') ms, launches $(grep 'part 0' gpurun_out/$1/rl$rl.log | tail -1 | awk '{print $NF}')"
done

# GPU-box: the bench's distributed path with two ranks on the one GPU (gloo fallback), short run
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist2}
mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench2.json 2> $OUT/bench2.log || { tail -30 $OUT/bench2.log; exit 1; }
cat $OUT/bench2.json

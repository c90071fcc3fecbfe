set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2g
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "comm or cfg3_strat or mouse_cov" > gpurun_out/r2g/pytest.log 2>&1 || { tail -30 gpurun_out/r2g/pytest.log; exit 1; }
tail -2 gpurun_out/r2g/pytest.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-grm > gpurun_out/r2g/bench2.json 2> gpurun_out/r2g/bench2.log; rc=$?
echo "2-rank rc=$rc"; tail -5 gpurun_out/r2g/bench2.log; cut -c1-600 gpurun_out/r2g/bench2.json

set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FEN_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --train-steps 3 \
    --no-stress > gpurun_out/dp2_bench.json 2> gpurun_out/dp2_bench.log
echo DP2_OK
tail -1 gpurun_out/dp2_bench.json

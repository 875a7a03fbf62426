# N=2 rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks share cuda:0 over
# gloo (RCCL refuses two ranks on one device); inference replicas + the DP training step, then
# the eager step's phases (tools/time_train_eager.py: step with / without the bucket exchange,
# bare all_reduce of the arena).  Timings are a rehearsal only: gloo stages CUDA tensors
# through the host and the two processes time-share the card.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FEN_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --train-steps 3 \
    --no-perceptual --no-stress > gpurun_out/dp2_bench.json 2> gpurun_out/dp2_bench.log
echo DP2_OK
FEN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29518 tools/time_train_eager.py > gpurun_out/dp2_eager.log 2>&1
echo EAGER_OK
tail -1 gpurun_out/dp2_bench.json
grep ms gpurun_out/dp2_eager.log

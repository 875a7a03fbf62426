# N=2 rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks share cuda:0 over
# gloo (RCCL refuses two ranks on one device); inference replicas + the DP training step.
# FEN_RCAB_FUSED=0: the fused RCAB needs all tiles of an image co-resident (its SE-gate hand-off
# spins on the other blocks), which two processes time-sharing one GPU do not guarantee.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FEN_RCAB_FUSED=0 FEN_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --train-steps 3 \
    --no-perceptual > gpurun_out/dp2_bench.log 2>&1 && echo DP2_OK
tail -1 gpurun_out/dp2_bench.log

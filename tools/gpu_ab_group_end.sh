# group-end fusion: the group / RCAB tests, the network-level parity tests, then same-box A/B
# of the inference bench and the training step
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ge.log 2>&1 || { tail -40 gpurun_out/pytest_ge.log; exit 1; }
tail -2 gpurun_out/pytest_ge.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_northstar.py tests/test_gpu_lite.py tests/test_gpu_dp_engine.py tests/test_gpu_perceptual_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ge2.log 2>&1 || { tail -40 gpurun_out/pytest_ge2.log; exit 1; }
tail -2 gpurun_out/pytest_ge2.log
AB_OFF="FEN_GROUP_END=split" AB_ON="FEN_GROUP_END=fused" REPS=3 bash tools/gpu_ab_env.sh
AB_CONFIGS="FEN_GROUP_END=split;FEN_GROUP_END=fused" REPS=2 bash tools/gpu_ab_train_env.sh

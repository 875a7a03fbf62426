# DOT epilogue: kernel tests, the training-parity tests, same-box A/B of the training step
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_dp_engine.py tests/test_gpu_rcab.py tests/test_gpu_lite.py tests/test_gpu_perceptual_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dot.log 2>&1 || { tail -30 gpurun_out/pytest_dot.log; exit 1; }
tail -2 gpurun_out/pytest_dot.log
AB_CONFIGS="FEN_SE_DOT=pass;FEN_SE_DOT=fused" REPS=3 bash tools/gpu_ab_train_env.sh

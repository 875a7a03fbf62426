# wgrad batching: kernel tests, the training-parity tests, then a same-box A/B of the
# graph-replayed stage-1 step over FEN_WGRAD_BATCH (1 = one launch per conv).
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad" tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_dp_engine.py tests/test_gpu_rcab.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_wg.log 2>&1 || { tail -30 gpurun_out/pytest_wg.log; exit 1; }
tail -2 gpurun_out/pytest_wg.log
AB_CONFIGS="FEN_WGRAD_BATCH=1;FEN_WGRAD_BATCH=2;FEN_WGRAD_BATCH=4;FEN_WGRAD_BATCH=8" REPS=2 bash tools/gpu_ab_train_env.sh

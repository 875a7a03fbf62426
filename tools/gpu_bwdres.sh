# a group's first RCAB on the fused backward (second residual in the DOT slot): parity, then a
# same-box A/B of FEN_RCAB_BWD_RES on the training step
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_bres.log 2>&1 || { tail -40 gpurun_out/pytest_bres.log; exit 1; }
tail -1 gpurun_out/pytest_bres.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_perceptual_train.py tests/test_gpu_northstar.py tests/test_gpu_lite.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_bres2.log 2>&1 || { tail -40 gpurun_out/pytest_bres2.log; exit 1; }
tail -1 gpurun_out/pytest_bres2.log
AB_CONFIGS="FEN_RCAB_BWD_RES=0;FEN_RCAB_BWD_RES=1" REPS=3 bash tools/gpu_ab_train_env.sh

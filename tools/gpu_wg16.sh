set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tks
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_perceptual_train.py tests/test_gpu_ssim.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_wg16.log 2>&1 || { tail -30 gpurun_out/pytest_wg16.log; exit 1; }
tail -2 gpurun_out/pytest_wg16.log
STEPS=30 timeout -k 10 300 python tools/train_step.py
AB_CONFIGS="FEN_WGRAD_BATCH=8" bash tools/gpu_train_kstats.sh
find gpurun_out/tks/c1 -name '*kernel_stats.csv' -exec cp {} gpurun_out/train_kstats.csv \;

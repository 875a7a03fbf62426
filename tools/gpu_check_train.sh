# full GPU test suite, then the per-kernel training breakdown (rocprofv3 stats of one config)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tks
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
AB_CONFIGS="${AB_CONFIGS:-FEN_WGRAD_BATCH=8}" bash tools/gpu_train_kstats.sh
cp gpurun_out/tks/c1/*/run_kernel_stats.csv gpurun_out/train_kstats.csv 2>/dev/null || find gpurun_out/tks/c1 -name '*kernel_stats.csv' -exec cp {} gpurun_out/train_kstats.csv \;

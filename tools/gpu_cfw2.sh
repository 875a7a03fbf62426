# conv_first weight gradient with block-reduced partials: parity, then per-kernel durations
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k conv_first -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_cfw2.log 2>&1 || { tail -40 gpurun_out/pytest_cfw2.log; exit 1; }
tail -2 gpurun_out/pytest_cfw2.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_disc.py tests/test_gpu_gan_step.py tests/test_gpu_lite.py tests/test_gpu_module.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cfw2b.log 2>&1 || { tail -40 gpurun_out/pytest_cfw2b.log; exit 1; }
tail -2 gpurun_out/pytest_cfw2b.log
bash tools/gpu_cf16_prof.sh

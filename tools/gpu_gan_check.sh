# discriminator / GAN parity tests (incl. the space-to-depth stride-2 kernels), then GAN timing
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k s2d -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gan.log 2>&1 || { tail -40 gpurun_out/pytest_gan.log; exit 1; }
tail -2 gpurun_out/pytest_gan.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_gan_step.py tests/test_gpu_gan_capture.py tests/test_gpu_trainer_resume.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gan.log 2>&1 || { tail -40 gpurun_out/pytest_gan.log; exit 1; }
tail -2 gpurun_out/pytest_gan.log
for r in 1 2 3; do timeout -k 10 300 python tools/gan_step.py | tail -1; done

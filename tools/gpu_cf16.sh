# conv_first forward on the split-f16 matrix cores: parity (conv_first kernels, VGG, D, net,
# GAN), then same-box A/B of FEN_CF_M16 on the perceptual step and the GAN iteration
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k conv_first -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_cf16.log 2>&1 || { tail -40 gpurun_out/pytest_cf16.log; exit 1; }
tail -2 gpurun_out/pytest_cf16.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_vgg.py tests/test_gpu_perceptual_train.py tests/test_gpu_net.py tests/test_gpu_disc.py tests/test_gpu_gan_step.py tests/test_gpu_lite.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cf16b.log 2>&1 || { tail -40 gpurun_out/pytest_cf16b.log; exit 1; }
tail -2 gpurun_out/pytest_cf16b.log
for r in 1 2; do
  for v in FEN_CF_M16=0 FEN_CF_M16=1; do
    echo "$v perceptual | $(env $v PERCEPTUAL=1 STEPS=20 timeout -k 10 300 python tools/train_step.py 2>/dev/null | tail -1)"
    echo "$v gan | $(env $v timeout -k 10 300 python tools/gan_step.py 2>/dev/null | tail -1)"
  done
done

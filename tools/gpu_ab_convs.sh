# streamed-conv variant (build_var/libfen_hip_$V.so) vs default: conv kernel tests on the
# variant, VGG conv shapes, the perceptual training step and the GAN iteration, same box
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VL="FEN_HIP_LIB=$GRAFT_REPO_ROOT/face-super-resolution_amd/csrc/build_var/libfen_hip_${V}.so"
env $VL timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_vgg.py tests/test_gpu_disc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_var.log 2>&1 || { tail -40 gpurun_out/pytest_var.log; exit 1; }
tail -2 gpurun_out/pytest_var.log
for r in 1 2; do
  for v in FEN_X=0 "$VL"; do
    echo "$v | vgg $(env $v timeout -k 10 200 python tools/bench_vgg_conv.py | tail -1 | cut -c1-400)"
    echo "$v | gan $(env $v timeout -k 10 300 python tools/gan_step.py | tail -1)"
  done
done

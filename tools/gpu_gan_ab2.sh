# HipAdamW with four float4 chunks per thread + the D head's forward GEMM reading its weight once
# for the pair pass (product) vs the previous commit's library (base): optimizer / head / D parity,
# then the GAN iteration, same box
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_optim.py tests/test_gpu_disc.py tests/test_gpu_bn_multi.py tests/test_gpu_gan_step.py tests/test_gpu_bench_legs.py" VARIANTS="prod" TEST_TIMEOUT=900 bash tools/gpu_ab.sh
VARIANTS="prod base" CMD="python tools/gan_step.py" CMD_ENV="STEPS=10" REPS=3 bash tools/gpu_ab.sh

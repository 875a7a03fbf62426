# the D step's real and fake batches as one discriminator pass (VGGStyleDiscriminator.forward_pair,
# per-batch BatchNorm statistics) vs two calls (FEN_D_PAIR=0): GAN parity tests, then the
# iteration time, same box, interleaved
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_gan_capture.py tests/test_gpu_gan_step.py tests/test_gpu_rccl.py tests/test_gpu_disc.py tests/test_gpu_bench_legs.py" VARIANTS="prod" TEST_TIMEOUT=900 bash tools/gpu_ab.sh
CONFIGS="FEN_D_PAIR=1;FEN_D_PAIR=0" CMD="python tools/gan_step.py" CMD_ENV="STEPS=10" REPS=3 bash tools/gpu_ab.sh

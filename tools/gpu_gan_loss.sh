# GANLoss on fen_gan_loss (one launch each way) vs the torch criteria (FEN_GAN_LOSS=0):
# GAN / discriminator parity, then the iteration time, same box
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_disc.py tests/test_gpu_gan_capture.py tests/test_gpu_gan_step.py tests/test_gpu_rccl.py tests/test_gpu_bench_legs.py" VARIANTS="prod" TEST_TIMEOUT=900 bash tools/gpu_ab.sh
CONFIGS="FEN_GAN_LOSS=1;FEN_GAN_LOSS=0" CMD="python tools/gan_step.py" CMD_ENV="STEPS=10" REPS=3 bash tools/gpu_ab.sh

# The pair pass's BatchNorm in one launch set for both batches (fen_bn_*_n) vs one per batch
# (FEN_D_BN_MULTI=0): grouped-vs-per-group bit-identity, GAN / discriminator parity, then the
# iteration time, same box
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_bn_multi.py tests/test_gpu_disc.py tests/test_gpu_gan_capture.py tests/test_gpu_gan_step.py tests/test_gpu_bench_legs.py" VARIANTS="prod" TEST_TIMEOUT=900 bash tools/gpu_ab.sh
CONFIGS="FEN_D_BN_MULTI=1;FEN_D_BN_MULTI=0" CMD="python tools/gan_step.py" CMD_ENV="STEPS=10" REPS=3 bash tools/gpu_ab.sh

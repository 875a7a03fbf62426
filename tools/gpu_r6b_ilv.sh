# round 6b: the wide conv's DMA pieces interleaved into the first MFMA half (product) vs issued
# before it (CVX_NO_ILV variant): parity on the product library, per-layer VGG conv times and
# the perceptual step, same box, interleaved
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_conv_wide.py tests/test_gpu_vgg.py tests/test_gpu_disc.py" VARIANTS="prod" bash tools/gpu_ab.sh
VARIANTS="prod noilv" CMD="python tools/bench_vgg_conv.py" REPS=2 bash tools/gpu_ab.sh
VARIANTS="prod noilv" CMD="python tools/train_step.py" CMD_ENV="PERCEPTUAL=1 STEPS=20" REPS=3 bash tools/gpu_ab.sh

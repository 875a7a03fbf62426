# round 6b: the wide conv's halo DMA in three bursts vs one (CVX_HALO_BURST variant): parity on the
# product library, then per-layer VGG conv times and the perceptual step, same box, interleaved
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_conv_wide.py tests/test_gpu_vgg.py tests/test_gpu_disc.py" VARIANTS="prod" bash tools/gpu_ab.sh
VARIANTS="prod burst" CMD="python tools/bench_vgg_conv.py" REPS=2 bash tools/gpu_ab.sh
VARIANTS="prod burst" CMD="python tools/train_step.py" CMD_ENV="PERCEPTUAL=1 STEPS=20" REPS=3 bash tools/gpu_ab.sh

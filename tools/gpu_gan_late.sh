# Late round-6 GAN changes (grouped BN passes, per-batch finalizes, the D head's single weight
# read) vs a base library built from an earlier commit (make ... OUT=build_var/libfen_hip_base.so):
# BN / D / GAN parity, the GAN iteration same box, then the configs[2] / configs[3] breakdowns
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_gpu_bn_multi.py tests/test_gpu_disc.py tests/test_gpu_optim.py tests/test_gpu_gan_capture.py tests/test_gpu_gan_step.py tests/test_gpu_bench_legs.py" VARIANTS="prod" TEST_TIMEOUT=900 bash tools/gpu_ab.sh
VARIANTS="prod base" CMD="python tools/gan_step.py" CMD_ENV="STEPS=10" REPS=3 bash tools/gpu_ab.sh
bash tools/gpu_r6_legprof.sh > gpurun_out/legprof.txt 2>&1
echo LEGPROF_OK

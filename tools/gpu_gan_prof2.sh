# the GAN iteration's kernel breakdown alone (rocprofv3 --kernel-trace --stats of tools/gan_step.py)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ganprof
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ganprof/gan -o run --output-format csv -- python tools/gan_step.py > gpurun_out/ganprof/gan.log 2>&1
tail -1 gpurun_out/ganprof/gan.log

# round 6 (second session) baseline: full GPU suite + smoke + bench on the restored tree, then a
# kernel trace (timestamps) of the perceptual step to place the copyBuffer blits in the sequence
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
mkdir -p gpurun_out/r6b
PERCEPTUAL=1 STEPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r6b/kt -o run --output-format csv -- python tools/train_step.py > gpurun_out/r6b/kt.log 2>&1
echo KT_OK

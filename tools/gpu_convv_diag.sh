set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
VARIANTS="prod now noh nobar noepi" CMD="python tools/bench_vgg_conv.py" REPS=2 bash tools/gpu_ab.sh

# same-box A/B: the folded SE backward's operand loads before the start-up DMA (default) or
# after it (SEB_LATE_LOADS variant), on the training step; fold parity on the variant first
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VL="FEN_HIP_LIB=$GRAFT_REPO_ROOT/face-super-resolution_amd/csrc/build_var/libfen_hip_late.so"
env $VL timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py -k se_fold -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_late.log 2>&1 || { tail -40 gpurun_out/pytest_late.log; exit 1; }
tail -1 gpurun_out/pytest_late.log
AB_CONFIGS="FEN_X=0;$VL;FEN_SE_IN_BWD=launch" REPS=3 bash tools/gpu_ab_train_env.sh

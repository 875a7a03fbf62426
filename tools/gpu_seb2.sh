# folded SE backward parity + train A/B (tools/gpu_seb.sh), then the RD_EARLY_GATE variant
# (the forward gate chain's operands issued before the start-up DMA): RCAB parity on the
# variant and a same-box inference / training A/B against the default library
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_seb.sh
VL="FEN_HIP_LIB=$GRAFT_REPO_ROOT/face-super-resolution_amd/csrc/build_var/libfen_hip_early.so"
env $VL timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_early.log 2>&1 || { tail -40 gpurun_out/pytest_early.log; exit 1; }
tail -1 gpurun_out/pytest_early.log
AB_OFF="FEN_X=0" AB_ON="$VL" REPS=2 bash tools/gpu_ab_env.sh
AB_CONFIGS="FEN_X=0;$VL" REPS=2 bash tools/gpu_ab_train_env.sh

# Same-box A/B of a variant library (face-super-resolution_amd/csrc/build_var/libfen_hip_$V.so,
# `make -C face-super-resolution_amd/csrc variant V=... DEFS=...`) against the default: the RCAB
# and network parity tests on the variant, then the inference bench and the training step.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VL="FEN_HIP_LIB=$GRAFT_REPO_ROOT/face-super-resolution_amd/csrc/build_var/libfen_hip_${V}.so"
env $VL timeout -k 10 600 python -u -m pytest tests/test_gpu_rcab.py tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_northstar.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_var.log 2>&1 || { tail -40 gpurun_out/pytest_var.log; exit 1; }
tail -2 gpurun_out/pytest_var.log
AB_OFF="FEN_X=0" AB_ON="$VL" REPS=3 bash tools/gpu_ab_env.sh
AB_CONFIGS="FEN_X=0;$VL" REPS=2 bash tools/gpu_ab_train_env.sh

# Upsampler stage-1 phase stamps (conv stamp library) + the bf16 strip-vs-per-RCAB training test.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/up
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_train64.py -k strip_vs_per_rcab > gpurun_out/up/t64.log 2>&1
echo "t64 rc=$?"; tail -5 gpurun_out/up/t64.log
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so UP=1 timeout -k 10 200 \
    python tools/stamp_conv.py > gpurun_out/up/stamps.txt 2>&1
echo "stamp rc=$?"; tail -40 gpurun_out/up/stamps.txt

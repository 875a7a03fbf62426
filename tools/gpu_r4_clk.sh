# In-kernel shader clock of k_group_strip (fp16 inference, after ~2 s of back-to-back forwards) and
# of the upsampler stage-1 conv (2 s of launches), from the two diagnostic stamp builds.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/clk
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 \
    python tools/stamp_strip.py > gpurun_out/clk/strip.txt 2>&1
echo "strip rc=$?"; cat gpurun_out/clk/strip.txt
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so UP=1 REPS=12000 timeout -k 10 200 \
    python tools/stamp_conv.py > gpurun_out/clk/up.txt 2>&1
echo "up rc=$?"; tail -3 gpurun_out/clk/up.txt
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
    tests/test_gpu_train64.py -k strip_vs_per_rcab > gpurun_out/clk/t64.log 2>&1
echo "t64 rc=$?"; grep -E "strip vs|passed|failed" gpurun_out/clk/t64.log

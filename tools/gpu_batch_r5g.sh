# round-5 batch g: the 128-channel conv1's gate operands (tile sums, FC1, FC2) by LDS-DMA ahead
# of the x / t staging (build_var/gate): its parity tests, then the stress leg A/B vs the product
export TMPDIR=/tmp
mkdir -p gpurun_out
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_gate.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rcab128.py > gpurun_out/t_gate.log 2>&1
rc=$?; echo "gate tests rc=$rc"; tail -2 gpurun_out/t_gate.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_gate.log | head -20; exit 1; }
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_gate.so; do
    FEN_HIP_LIB=$l STEPS=5 timeout -k 10 300 python tools/stress_step.py > gpurun_out/st.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "stress $l rc=$rc"; tail -5 gpurun_out/st.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/st.log)"
  done
done

# round-5 batch h: the streamed conv's pipelined tap (k-half 1 and the next tap's halo fragments
# read under the current MFMAs; the halo prefetch at 6 chunks per tap pipeline, build_var/pipe6)
# vs the product: tests with the variant, then the training A/B and op times
export TMPDIR=/tmp
mkdir -p gpurun_out
V=face-super-resolution_amd/csrc/build_var/libfen_hip_pipe6.so
FEN_HIP_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train64.py > gpurun_out/t_h.log 2>&1
rc=$?; echo "pipe6 tests rc=$rc"; tail -2 gpurun_out/t_h.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_h.log | head -20; exit 1; }
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so $V; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done
FEN_HIP_LIB=$V TRAIN=1 REPS=10 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train_h.txt 2>&1
echo "op_times rc=$?"; grep -E "256->64|sum of" gpurun_out/ops_train_h.txt

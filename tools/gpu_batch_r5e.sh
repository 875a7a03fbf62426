# round-5 batch e: k_cl_bwd with its P^T chunks swizzled (the transposed writes were 8-way bank
# conflicts) in the product; build_var/epf adds the conv epilogue's PRELU_BWD / DOT operands
# prefetched for the whole tile; build_var/noswz is the previous product.  Tests first, then the
# training A/B and op times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv_last" > gpurun_out/t_cl.log 2>&1
rc=$?; echo "conv_last tests rc=$rc"; tail -2 gpurun_out/t_cl.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_cl.log | head -20; exit 1; }
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_epf.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train64.py > gpurun_out/t_epf.log 2>&1
rc=$?; echo "epf tests rc=$rc"; tail -2 gpurun_out/t_epf.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_epf.log | head -20; exit 1; }
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_noswz.so face-super-resolution_amd/csrc/build_var/libfen_hip_epf.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done
TRAIN=1 REPS=10 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train.txt 2>&1
echo "op_times rc=$?"; grep -E "conv_last|256->64|sum of" gpurun_out/ops_train.txt
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_epf.so TRAIN=1 REPS=10 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train_epf.txt 2>&1
echo "op_times epf rc=$?"; grep -E "conv_last|256->64|sum of" gpurun_out/ops_train_epf.txt

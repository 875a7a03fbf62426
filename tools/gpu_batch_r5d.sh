# round-5 batch d: the fused conv_last backward after the scratch fix (its im2col k half made a
# template constant) and the streamed conv's two-step weight pipeline: kernel + training tests,
# A/B against FEN_CL_BWD=0 and against the streamed conv without the pipeline (build_var/nopf),
# op times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train64.py > gpurun_out/t_cl.log 2>&1
rc=$?; echo "conv_last tests rc=$rc"; tail -2 gpurun_out/t_cl.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_cl.log | head -20; exit 1; }
for rep in 1 2 3; do
  for v in 1 0; do
    FEN_CL_BWD=$v STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train CL_BWD=$v rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "CL_BWD=$v   $(tail -1 gpurun_out/ab_t.log)"
  done
done
for rep in 1 2; do
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_nopf.so STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
  echo "nopf   $(tail -1 gpurun_out/ab_t.log)"
done
TRAIN=1 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train.txt 2>&1
echo "op_times rc=$?"; grep -E "conv_last|conv3x3 .*256->64|sum of" gpurun_out/ops_train.txt
FEN_CL_BWD=0 TRAIN=1 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train0.txt 2>&1
echo "op_times0 rc=$?"; grep -E "conv_last|wgrad3x3 .*64->16|wgrad3x3 .*->16|sum of" gpurun_out/ops_train0.txt

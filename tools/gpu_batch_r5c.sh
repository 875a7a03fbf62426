# round-5 batch c: the kernel tests first (the fused conv_last backward k_cl_bwd, the persistent
# conv_last dgrad k_cld_p, the streamed conv's next-panel halo prefetch), then the strip-backward per-strip dalpha and training-path tests, the
# fc2e variant's forward parity, then the training A/B (fused tail backward vs FEN_CL_BWD=0) and
# the inference A/B (fc2e), op times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/t_cl.log 2>&1
rc=$?; echo "conv_last tests rc=$rc"; tail -3 gpurun_out/t_cl.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_cl.log | head -20; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_strip_bwd.py tests/test_gpu_train64.py tests/test_gpu_strip_status.py tests/test_gpu_rccl.py > gpurun_out/t_prod.log 2>&1
rc=$?; echo "product tests rc=$rc"; tail -2 gpurun_out/t_prod.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_prod.log | head -20; exit 1; }
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_fc2e.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_chain.py tests/test_gpu_group_strip.py > gpurun_out/t_fc2e.log 2>&1
rc=$?; echo "fc2e tests rc=$rc"; tail -2 gpurun_out/t_fc2e.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    FEN_CL_BWD=$v STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train CL_BWD=$v rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "CL_BWD=$v   $(tail -1 gpurun_out/ab_t.log)"
  done
done
INF=1 REPS=2 bash tools/gpu_ab_r5.sh
timeout -k 10 200 python tools/op_times.py > gpurun_out/ops_inf.txt 2>&1
TRAIN=1 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train.txt 2>&1
echo "op_times rc=$?"

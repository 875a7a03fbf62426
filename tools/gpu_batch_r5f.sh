# round-5 batch f: tests of the product (conv_last backward swizzle, conv epilogue operand
# prefetch, SSIM two-launch form), the SSIM timing (one launch vs two), then the training A/B
# against build_var/noswz (-DCLB_NOSWZ) and build_var/noepf (-DEPI_NOPF), op times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_ssim.py tests/test_gpu_train64.py > gpurun_out/t_f.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_f.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_f.log | head -20; exit 1; }
timeout -k 10 120 python tools/bench_ssim.py > gpurun_out/ssim_f.json 2> gpurun_out/ssim_f.err
echo "bench_ssim rc=$? $(cat gpurun_out/ssim_f.json)"
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_noswz.so face-super-resolution_amd/csrc/build_var/libfen_hip_noepf.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done
TRAIN=1 REPS=10 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train.txt 2>&1
echo "op_times rc=$?"; grep -E "conv_last|256->64|sum of" gpurun_out/ops_train.txt

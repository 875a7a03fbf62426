# one box: training parity tests + the strip-backward weight-gradient batch A/B, then the
# stagger variant's strip parity tests + the inference A/B (tools/gpu_ab_strip.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train64.py tests/test_gpu_group_strip_bwd.py tests/test_gpu_module.py tests/test_gpu_net.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/trainpar.log 2>&1
rc=$?; tail -3 gpurun_out/trainpar.log; [ $rc -eq 0 ] || exit 1
AB_CONFIGS="FEN_WGRAD_STRIP_BATCH=8;FEN_WGRAD_STRIP_BATCH=32" REPS=3 bash tools/gpu_ab_train_env.sh || exit 1
for l in face-super-resolution_amd/csrc/build_var/libfen_hip_*.so; do
  FEN_HIP_LIB=$l timeout -k 10 300 python -u -m pytest tests/test_gpu_group_strip.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var_tests.log 2>&1
  rc=$?; echo "$l tests rc=$rc"; tail -2 gpurun_out/var_tests.log; [ $rc -eq 0 ] || exit 1
done
bash tools/gpu_ab_strip.sh

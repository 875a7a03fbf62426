# DP capture (one-rank RCCL), GAN capture, DP engine stand-in, group strip, north-star training parity
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_gan_capture.py tests/test_gpu_dp_engine.py tests/test_gpu_group_strip.py tests/test_gpu_train64.py -m gpu -v -s -x --timeout 300 --timeout-method thread > gpurun_out/dp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error|worst|rel " gpurun_out/dp_tests.log | tail -40
exit $rc

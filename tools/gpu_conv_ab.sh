set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv3x3 or dgrad or upsample" --timeout 120 --timeout-method thread > gpurun_out/conv_pytest.log 2>&1 || { tail -30 gpurun_out/conv_pytest.log; exit 1; }
tail -1 gpurun_out/conv_pytest.log
timeout -k 10 120 python tools/bench_conv.py
FEN_CONV_VARIANT=5 timeout -k 10 120 python tools/bench_conv.py

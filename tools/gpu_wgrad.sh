set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/wgrad_pytest.log 2>&1 || { tail -30 gpurun_out/wgrad_pytest.log; exit 1; }
tail -2 gpurun_out/wgrad_pytest.log
timeout -k 10 120 python tools/bench_conv.py
FEN_WGRAD_OLD=1 timeout -k 10 120 python tools/bench_conv.py

set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/t6.log 2>&1 || { tail -40 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
timeout -k 10 120 python tools/bench_conv.py
FEN_WGRAD_KH3=1 timeout -k 10 120 python tools/bench_conv.py

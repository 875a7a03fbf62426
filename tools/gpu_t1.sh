set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rcab.py tests/test_gpu_module.py tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1
timeout -k 10 120 python tools/bench_conv.py

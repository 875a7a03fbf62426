set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "conv_first or conv_last" -x -q --timeout 120 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -40 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log

timeout -k 10 60 python tools/bench_last.py

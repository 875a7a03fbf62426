set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_strip_status.py tests/test_gpu_group_strip.py tests/test_gpu_group_strip_bwd.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_status.log 2>&1 || { tail -60 gpurun_out/t_status.log; exit 1; }
tail -3 gpurun_out/t_status.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log && echo BENCH_OK
tail -1 gpurun_out/bench.json

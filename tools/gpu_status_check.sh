# round-4 checks: strip status word (fault injection), strip kernels, the bench legs at bench size, bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_strip_status.py tests/test_gpu_bench_legs.py tests/test_gpu_group_strip.py tests/test_gpu_group_strip_bwd.py -v -s --timeout 300 --timeout-method thread > gpurun_out/t_status.log 2>&1 || { tail -80 gpurun_out/t_status.log; exit 1; }
grep -E "passed|failed|B=|bf16|GAN|gradients" gpurun_out/t_status.log | tail -20
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log && echo BENCH_OK
tail -1 gpurun_out/bench.json

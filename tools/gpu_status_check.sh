# round-4 checks: the GAN leg at D input 256, then the bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_legs.py -k gan_leg_d256 -v -s --timeout 300 --timeout-method thread > gpurun_out/t_gan.log 2>&1 || { tail -40 gpurun_out/t_gan.log; exit 1; }
grep -E "passed|failed|GAN|gradients" gpurun_out/t_gan.log | tail -8
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log && echo BENCH_OK
tail -1 gpurun_out/bench.json

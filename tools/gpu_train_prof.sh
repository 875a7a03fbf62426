# training-step kernel stats (bench training leg only) + the SE-backward kernel tests
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rcab.py tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tp/pytest.log 2>&1 || { tail -30 gpurun_out/tp/pytest.log; exit 1; }
tail -1 gpurun_out/tp/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp/p -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/tp/bench.log 2>&1
python tools/prof_summary.py stats "$(find gpurun_out/tp/p -name '*kernel_stats.csv' | head -1)" gpurun_out/tp/stats.csv | head -20
tail -1 gpurun_out/tp/bench.log | cut -c1-200

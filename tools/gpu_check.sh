set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK
tail -1 gpurun_out/bench.log

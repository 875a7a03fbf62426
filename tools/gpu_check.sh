# full GPU check: parity tests, smoke, bench (one line of JSON at the end)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log && echo BENCH_OK
tail -1 gpurun_out/bench.json

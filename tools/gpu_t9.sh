set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py tests/test_gpu_module.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t9.log 2>&1 || { tail -40 gpurun_out/t9.log; exit 1; }
tail -1 gpurun_out/t9.log
VARIANTS="${VARIANTS:-div noprio}" bash tools/gpu_ab_rcab.sh

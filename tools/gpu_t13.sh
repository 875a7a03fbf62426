set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_module.py tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t13.log 2>&1 || { tail -40 gpurun_out/t13.log; exit 1; }
tail -1 gpurun_out/t13.log
timeout -k 10 60 python tools/bench_last.py
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_base.so timeout -k 10 60 python tools/bench_last.py

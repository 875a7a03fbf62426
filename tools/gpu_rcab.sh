set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rcab_pytest.log 2>&1 || { tail -40 gpurun_out/rcab_pytest.log; exit 1; }
tail -1 gpurun_out/rcab_pytest.log
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so timeout -k 10 120 python -u tools/stamp_rcab.py
timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1
timeout -k 10 120 python tools/bench_conv.py

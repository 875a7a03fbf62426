set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py tests/test_gpu_module.py tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t12.log 2>&1 || { tail -40 gpurun_out/t12.log; exit 1; }
tail -1 gpurun_out/t12.log
VARIANTS="${VARIANTS:-base}" bash tools/gpu_ab_rcab.sh
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so timeout -k 10 120 python -u tools/stamp_rcab.py | tail -1

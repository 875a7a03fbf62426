set -e
export TMPDIR=/tmp
FEN_CONV_VARIANT=4 timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_net.py tests/test_gpu_module.py -q -x > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -1 gpurun_out/q_pytest.log
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so B=32 FEN_CONV_VARIANT=4 timeout -k 10 120 python tools/stamp_conv.py
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so B=128 FEN_CONV_VARIANT=4 timeout -k 10 120 python tools/stamp_conv.py
FEN_CONV_VARIANT=4 timeout -k 10 300 python tools/bench_conv.py
FEN_CONV_VARIANT=4 timeout -k 10 300 python bench.py --no-cpu-baseline

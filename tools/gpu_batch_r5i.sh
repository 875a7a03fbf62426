# round-5 batch i: the ping-pong conv's service phase without the DMA wait before its epilogue
# when the epilogue loads nothing (build_var/gnowait): tests with the variant, then the inference
# and training A/B against the product
export TMPDIR=/tmp
mkdir -p gpurun_out
V=face-super-resolution_amd/csrc/build_var/libfen_hip_gnowait.so
FEN_HIP_LIB=$V timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_northstar.py > gpurun_out/t_i.log 2>&1
rc=$?; echo "gnowait tests rc=$rc"; tail -2 gpurun_out/t_i.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_i.log | head -20; exit 1; }
INF=1 REPS=3 bash tools/gpu_ab_r5.sh

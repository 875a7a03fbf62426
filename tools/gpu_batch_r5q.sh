# round-5 batch q: fen_ssim_ex as one pipelined launch (k_ssim_pipe) vs build_var/nopipe (two
# launches), lag8 (8 images of lag), nowait (timing only: gradient blocks do not wait): SSIM
# tests on the product, bench_ssim A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ssim.py > gpurun_out/t_q.log 2>&1
rc=$?; echo "ssim tests rc=$rc"; tail -2 gpurun_out/t_q.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_q.log | head; exit 1; }
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_nopipe.so face-super-resolution_amd/csrc/build_var/libfen_hip_lag8.so face-super-resolution_amd/csrc/build_var/libfen_hip_nowait.so; do
    FEN_HIP_LIB=$l timeout -k 10 120 python tools/bench_ssim.py > gpurun_out/ab_s.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ssim $l rc=$rc"; tail -5 gpurun_out/ab_s.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_s.log)"
  done
done

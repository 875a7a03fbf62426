# round-5 batch s: SSIM two-launch form variants -- build_var/fullpix (k_ssim_g2 reads and writes
# whole 32-B pixels: full-sector stores), mapf16 (a / b / c maps as fp16), both -- SSIM tests on
# each variant, then bench_ssim A/B vs the product (3 reps)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in fullpix mapf16 both; do
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ssim.py > gpurun_out/t_s_$v.log 2>&1
  rc=$?; echo "$v ssim tests rc=$rc"; tail -1 gpurun_out/t_s_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_s_$v.log | head -5; [ $rc -eq 1 ] || exit $rc; }
done
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_fullpix.so face-super-resolution_amd/csrc/build_var/libfen_hip_mapf16.so face-super-resolution_amd/csrc/build_var/libfen_hip_both.so; do
    FEN_HIP_LIB=$l timeout -k 10 120 python tools/bench_ssim.py > gpurun_out/ab_s.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ssim $l rc=$rc"; tail -5 gpurun_out/ab_s.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_s.log)"
  done
done

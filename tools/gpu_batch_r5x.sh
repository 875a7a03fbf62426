# round-5 batch x: the SSIM map kernel's occupancy -- build_var/alias (horizontal sums over the
# staged inputs: 27.7 KB LDS, still 163 VGPRs), cb1 (fen_ssim_ex's first half one block per (tile,
# channel): 109 VGPRs, 42 KB), cb1a (both: 92 VGPRs, 27.7 KB -> 5 blocks per CU) vs the product:
# SSIM tests on each variant, then bench_ssim A/B (3 reps)
export TMPDIR=/tmp
mkdir -p gpurun_out
V=face-super-resolution_amd/csrc/build_var
for v in alias cb1 cb1a; do
  FEN_HIP_LIB=$V/libfen_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ssim.py > gpurun_out/t_x_$v.log 2>&1
  rc=$?; echo "$v ssim tests rc=$rc"; tail -1 gpurun_out/t_x_$v.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/t_x_$v.log | head -5; exit $rc; }
done
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so $V/libfen_hip_alias.so $V/libfen_hip_cb1.so $V/libfen_hip_cb1a.so; do
    FEN_HIP_LIB=$l timeout -k 10 120 python tools/bench_ssim.py > gpurun_out/ab_s.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ssim $l rc=$rc"; tail -5 gpurun_out/ab_s.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_s.log)"
  done
done

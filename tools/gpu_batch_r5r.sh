# round-5 batch r: SSIM LDS layouts -- build_var/ssimA (the horizontal sums as (mp, mt) / (E[p^2],
# E[t^2]) pairs: 8-B LDS accesses straight into the packed FMAs' operands), ssimB (+ the inputs as
# (p, t) pairs) vs the product: SSIM tests on both variants, then bench_ssim A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ssimA ssimB; do
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ssim.py > gpurun_out/t_r_$v.log 2>&1
  rc=$?; echo "$v ssim tests rc=$rc"; tail -1 gpurun_out/t_r_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_r_$v.log | head; exit 1; }
done
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_ssimA.so face-super-resolution_amd/csrc/build_var/libfen_hip_ssimB.so; do
    FEN_HIP_LIB=$l timeout -k 10 120 python tools/bench_ssim.py > gpurun_out/ab_s.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ssim $l rc=$rc"; tail -5 gpurun_out/ab_s.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_s.log)"
  done
done

# round-5 batch m: cache-policy factorial on one box (batch j's box: saves nt -84 us; batch l's
# box: all three nt +100 us vs none).  cacheold = none, s = saves, sl = saves + bwd loads,
# sb = saves + dt / dz1 stores, product = all three.  Training A/B only (the variants differ
# in store / load policy bits, results bit-identical; batch l ran the tests on product/cacheold)
export TMPDIR=/tmp
mkdir -p gpurun_out
V=face-super-resolution_amd/csrc/build_var
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so $V/libfen_hip_cacheold.so $V/libfen_hip_s.so $V/libfen_hip_sl.so $V/libfen_hip_sb.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done

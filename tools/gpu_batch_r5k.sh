# round-5 batch k: the product now stores the training forward's saves non-temporal; variants:
# build_var/loadnt (the strip backward's loads of those saves non-temporal), build_var/bwsave
# (its dt / dz1 stores for the weight gradients non-temporal).  Tests, then the training A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train64.py tests/test_gpu_group_strip_bwd.py > gpurun_out/t_k.log 2>&1
rc=$?; echo "product tests rc=$rc"; tail -2 gpurun_out/t_k.log; [ $rc -eq 0 ] || exit 1
for v in loadnt bwsave; do
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train64.py > gpurun_out/t_k_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_loadnt.so face-super-resolution_amd/csrc/build_var/libfen_hip_bwsave.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done

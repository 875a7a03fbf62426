# round-5 batch l: the product (non-temporal training saves, strip-backward loads and dt / dz1
# stores) vs build_var/cacheold (all three plain, the round's earlier product) and
# build_var/wgnt (+ the persistent wgrad's operand DMA non-temporal): tests, then the training A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train64.py tests/test_gpu_group_strip_bwd.py tests/test_gpu_kernels.py -k "wgrad or train or strip" > gpurun_out/t_l.log 2>&1
rc=$?; echo "product tests rc=$rc"; tail -2 gpurun_out/t_l.log; [ $rc -eq 0 ] || exit 1
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_wgnt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train64.py tests/test_gpu_kernels.py -k "wgrad or train" > gpurun_out/t_l_wgnt.log 2>&1
rc=$?; echo "wgnt tests rc=$rc"; tail -2 gpurun_out/t_l_wgnt.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_cacheold.so face-super-resolution_amd/csrc/build_var/libfen_hip_wgnt.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done

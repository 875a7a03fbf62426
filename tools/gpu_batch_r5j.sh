# round-5 batch j: the training forward's saves as non-temporal stores (build_var/savent: the
# backward reads them ~ms later; plain stores allocate them in L2 / MALL beside the strip
# kernel's hand-off rows and filter taps): tests with the variant, then the training A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
V=face-super-resolution_amd/csrc/build_var/libfen_hip_savent.so
FEN_HIP_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train64.py tests/test_gpu_group_chain.py > gpurun_out/t_j.log 2>&1
rc=$?; echo "savent tests rc=$rc"; tail -2 gpurun_out/t_j.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_j.log | head -20; exit 1; }
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so $V; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done

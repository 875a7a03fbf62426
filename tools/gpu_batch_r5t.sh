# round-5 batch t: (1) SSIM two-launch variants (batch s: fullpix / mapf16 / both) -- tests on
# each, bench_ssim A/B; (2) strip backward SE sweep 8 granules at a time (product: no VGPR spill)
# vs build_var/poll16 (16 loads in flight, 9 VGPRs spilled to scratch) -- strip bwd tests on the
# product, then the training step A/B (3 reps)
export TMPDIR=/tmp
mkdir -p gpurun_out
V=face-super-resolution_amd/csrc/build_var
bash tools/gpu_batch_r5s.sh || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_group_strip_bwd.py tests/test_gpu_train64.py > gpurun_out/t_t.log 2>&1
rc=$?; echo "strip bwd / train64 tests rc=$rc"; tail -1 gpurun_out/t_t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_t.log | head -5; exit $rc; }
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so $V/libfen_hip_poll16.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done

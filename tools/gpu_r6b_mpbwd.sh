# round 6b: FEN_EPI_MAXPOOL_BWD -- parity (conv + VGG tests, bench legs' perceptual tests), then the
# perceptual step vs FEN_VGG_LEGACY=1 (round 5's VGG form) on the same box, then its kernel trace
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv_wide.py tests/test_gpu_vgg.py tests/test_gpu_perceptual_train.py tests/test_abi.py > gpurun_out/r6c/t1.log 2>&1 || { tail -30 gpurun_out/r6c/t1.log; exit 1; }
tail -1 gpurun_out/r6c/t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_legs.py -k "perceptual" > gpurun_out/r6c/t2.log 2>&1 || { tail -30 gpurun_out/r6c/t2.log; exit 1; }
tail -1 gpurun_out/r6c/t2.log
for rep in 1 2 3; do
  echo "new    $(PERCEPTUAL=1 STEPS=20 timeout -k 10 120 python tools/train_step.py)"
  echo "legacy $(FEN_VGG_LEGACY=1 PERCEPTUAL=1 STEPS=20 timeout -k 10 120 python tools/train_step.py)"
done
PERCEPTUAL=1 STEPS=4 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6c/kt -o run --output-format csv -- python tools/train_step.py > gpurun_out/r6c/kt.log 2>&1
echo KT_OK

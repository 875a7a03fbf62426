# round 6: k_conv3x3_v (the DMA-fed wide conv) -- parity first (a fault ends the call), then the
# VGG shapes A/B (variants from make variant), the perceptual / GAN steps against the streamed kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/convv
V=face-super-resolution_amd/csrc/build_var
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_wide.py > gpurun_out/convv/t_wide.log 2>&1
rc=$?; echo "wide tests rc=$rc: $(tail -1 gpurun_out/convv/t_wide.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/convv/t_wide.log | head -20; exit $rc; }
for l in ${VARIANTS:-}; do
  FEN_HIP_LIB=$V/libfen_hip_$l.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_wide.py > gpurun_out/convv/t_wide_$l.log 2>&1
  rc=$?; echo "$l wide tests rc=$rc: $(tail -1 gpurun_out/convv/t_wide_$l.log)"
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_vgg.py tests/test_gpu_perceptual_train.py tests/test_gpu_disc.py tests/test_gpu_gan_step.py tests/test_gpu_gan_capture.py tests/test_gpu_rccl.py tests/test_gpu_bench_legs.py > gpurun_out/convv/t_legs.log 2>&1
rc=$?; echo "leg tests rc=$rc: $(tail -1 gpurun_out/convv/t_legs.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/convv/t_legs.log | head -20; exit $rc; }
for rep in 1 2; do
  for l in prod ${VARIANTS:-} ${TIMEONLY:-}; do
    if [ $l = prod ]; then L=face-super-resolution_amd/src/hip/libfen_hip.so; else L=$V/libfen_hip_$l.so; fi
    FEN_HIP_LIB=$L timeout -k 10 120 python tools/bench_vgg_conv.py > gpurun_out/convv/vgg.txt 2>&1 || { tail -3 gpurun_out/convv/vgg.txt; exit 1; }
    echo "$l $(tail -1 gpurun_out/convv/vgg.txt)"
  done
done
FEN_CONV_V=0 timeout -k 10 120 python tools/bench_vgg_conv.py > gpurun_out/convv/vgg.txt 2>&1 && echo "streamed $(tail -1 gpurun_out/convv/vgg.txt)"
for rep in 1 2; do for v in 0 1; do
  FEN_CONV_V=$v PERCEPTUAL=1 STEPS=20 timeout -k 10 200 python tools/train_step.py > gpurun_out/convv/ts.log 2>&1 || { tail -5 gpurun_out/convv/ts.log; exit 1; }
  echo "FEN_CONV_V=$v perceptual $(tail -1 gpurun_out/convv/ts.log)"
done; done
for v in 0 1; do FEN_CONV_V=$v STEPS=5 timeout -k 10 300 python tools/gan_step.py > gpurun_out/convv/gan.log 2>&1 || { tail -5 gpurun_out/convv/gan.log; exit 1; }; echo "FEN_CONV_V=$v $(tail -1 gpurun_out/convv/gan.log)"; done

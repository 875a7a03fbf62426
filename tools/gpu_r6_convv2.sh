# round 6: wide conv parity (unrolled form) + the perceptual / GAN steps with it on / off + their profiles
export TMPDIR=/tmp
mkdir -p gpurun_out/convv2
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_conv_wide.py tests/test_gpu_vgg.py tests/test_gpu_perceptual_train.py tests/test_gpu_disc.py tests/test_gpu_bench_legs.py > gpurun_out/convv2/t.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/convv2/t.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/convv2/t.log | head -20; exit $rc; }
for rep in 1 2; do for v in 0 1; do
  FEN_CONV_V=$v PERCEPTUAL=1 STEPS=20 timeout -k 10 200 python tools/train_step.py > gpurun_out/convv2/ts.log 2>&1 || { tail -5 gpurun_out/convv2/ts.log; exit 1; }
  echo "FEN_CONV_V=$v perceptual $(tail -1 gpurun_out/convv2/ts.log)"
done; done
for rep in 1 2; do for v in 0 1; do FEN_CONV_V=$v STEPS=8 timeout -k 10 300 python tools/gan_step.py > gpurun_out/convv2/gan.log 2>&1 || { tail -5 gpurun_out/convv2/gan.log; exit 1; }; echo "FEN_CONV_V=$v $(tail -1 gpurun_out/convv2/gan.log)"; done; done
PERCEPTUAL=1 STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/convv2/perc -o run --output-format csv -- python tools/train_step.py > gpurun_out/convv2/perc.log 2>&1 || exit 1
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/convv2/gan -o run --output-format csv -- python tools/gan_step.py > gpurun_out/convv2/ganp.log 2>&1 || exit 1

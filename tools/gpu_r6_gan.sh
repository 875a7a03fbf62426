# round 6: the GAN iteration's HIP head / HipAdamW parity, then its timing and kernel breakdown
export TMPDIR=/tmp
mkdir -p gpurun_out/gan6
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_l1.py tests/test_gpu_disc.py tests/test_gpu_gan_step.py tests/test_gpu_gan_capture.py tests/test_gpu_rccl.py tests/test_gpu_trainer_resume.py tests/test_gpu_bench_legs.py > gpurun_out/gan6/t.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/gan6/t.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/gan6/t.log | head -20; exit $rc; }
for rep in 1 2; do STEPS=8 timeout -k 10 300 python tools/gan_step.py > gpurun_out/gan6/gan.log 2>&1 || { tail -5 gpurun_out/gan6/gan.log; exit 1; }; echo "$(tail -1 gpurun_out/gan6/gan.log)"; done
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gan6/prof -o run --output-format csv -- python tools/gan_step.py > gpurun_out/gan6/ganp.log 2>&1 || exit 1

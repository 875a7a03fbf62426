# round-5 batch u: SSIM two-launch form with fp16 maps for a bf16 gradient (tests + bench_ssim),
# the bench-config GAN bf16-vs-fp32 test, then the full GPU check (suite, smoke, bench line)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_ssim.py > gpurun_out/t_u_ssim.log 2>&1
rc=$?; echo "ssim tests rc=$rc"; grep -E "base|passed|failed" gpurun_out/t_u_ssim.log | tail -14; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/t_u_ssim.log | head -5; exit $rc; }
for rep in 1 2; do timeout -k 10 120 python tools/bench_ssim.py 2>/dev/null | tail -1; done
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_gpu_bench_legs.py -k bf16_vs_fp32 > gpurun_out/t_gan16.log 2>&1
rc=$?; echo "gan bf16 test rc=$rc"; grep -E "GAN bench|passed|failed|Error" gpurun_out/t_gan16.log | head -5
bash tools/gpu_check.sh

# round-5 batch v: the forward strip kernels' gate sweep 8 granules at a time (product) vs
# build_var/gpoll16 (16 loads per round): strip / chain / north-star tests on the product, the
# inference + training A/B (3 reps), then profiles of the late tree: SSIM op kernel stats
# (bench_ssim under rocprofv3) and the stage-1 training step's kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="tests/test_gpu_group_strip.py tests/test_gpu_group_chain.py tests/test_gpu_northstar.py" INF=1 REPS=3 bash tools/gpu_ab_r5.sh || exit $?
mkdir -p gpurun_out/pssim
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pssim -o run --output-format csv -- python tools/bench_ssim.py > gpurun_out/pssim/log.txt 2>&1
echo "ssim prof rc=$?"
f=$(find gpurun_out/pssim -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" gpurun_out/ssim_kernel_stats.csv && head -6 "$f" | cut -c1-160
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_X=0" bash tools/gpu_train_kstats.sh > gpurun_out/tks/summary.txt 2>&1
cat gpurun_out/tks/summary.txt
find gpurun_out/tks/c1 -name '*kernel_stats.csv' -exec cp {} gpurun_out/train_kstats.csv \;

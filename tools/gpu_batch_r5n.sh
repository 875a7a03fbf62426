# round-5 batch n: the two-launch SSIM's kernels separately (rocprofv3 kernel stats of bench_ssim)
export TMPDIR=/tmp
mkdir -p gpurun_out/ssimn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ssimn/prof -o run -- python tools/bench_ssim.py > gpurun_out/ssimn/bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/ssimn/bench.log; [ $rc -eq 0 ] || exit 1
find gpurun_out/ssimn/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/ssimn/kernel_stats.csv \;
cut -d, -f1-8 gpurun_out/ssimn/kernel_stats.csv | head -12

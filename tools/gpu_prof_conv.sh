# per-kernel stats of the conv/wgrad microbench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pc -o run --output-format csv -- python tools/bench_conv.py > gpurun_out/pc/log.txt 2>&1
python tools/prof_summary.py stats gpurun_out/pc/run_kernel_stats.csv gpurun_out/pc/stats.csv

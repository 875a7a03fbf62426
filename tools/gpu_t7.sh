set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/wg
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wg/a -o run --output-format csv -- python tools/bench_conv.py > gpurun_out/wg/a.log 2>&1
FEN_WGRAD_NKH1=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wg/b -o run --output-format csv -- python tools/bench_conv.py > gpurun_out/wg/b.log 2>&1
for v in a b; do f=$(find gpurun_out/wg/$v -name '*kernel_stats.csv' | head -1); grep -E "wgrad" $f | cut -c1-200; done

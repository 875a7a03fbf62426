# round-5 late check on the final tree: full GPU suite, smoke, bench line (tools/gpu_check.sh),
# then the bench's inference leg under rocprofv3 --kernel-trace --stats (the dominant launch's
# average for the roofline cross-check)
export TMPDIR=/tmp
mkdir -p gpurun_out/proff
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proff/inf -o run --output-format csv -- \
    python bench.py --no-train --no-stress --no-cpu-baseline > gpurun_out/proff/inf_bench.json 2> gpurun_out/proff/inf_bench.log
echo "inf prof rc=$?"
f=$(find gpurun_out/proff/inf -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" gpurun_out/inf_kernel_stats.csv && head -5 "$f" | cut -c1-150
tail -1 gpurun_out/proff/inf_bench.json | cut -c1-400

# BASELINE configs[4] (128 ch, 10x20 RCAB, x8, B=4, fp16 inference) under rocprofv3
# --kernel-trace --stats: per-kernel breakdown -> gpurun_out/stress/stress_kernel_stats.csv
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stress
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stress/p -o run --output-format csv -- python tools/stress_step.py > gpurun_out/stress/run.log 2>&1
tail -1 gpurun_out/stress/run.log
python tools/prof_summary.py stats "$(find gpurun_out/stress/p -name '*kernel_stats.csv' | head -1)" gpurun_out/stress/stress_kernel_stats.csv

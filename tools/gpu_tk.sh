set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_RCAB_BWD=fused" bash tools/gpu_train_kstats.sh
find gpurun_out/tks/c1 -name '*kernel_stats.csv' -exec cp {} gpurun_out/train_kstats.csv \;

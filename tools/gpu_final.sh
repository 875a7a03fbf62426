# round-end sequence: full GPU suite, smoke, bench, then the training step's kernel breakdown
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_X=0" bash tools/gpu_train_kstats.sh > gpurun_out/tks/summary.txt 2>&1
find gpurun_out/tks/c1 -name '*kernel_stats.csv' -exec cp {} gpurun_out/train_kstats.csv \;
head -5 gpurun_out/tks/summary.txt

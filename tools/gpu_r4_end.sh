# Round-4 end run: full GPU suite + smoke + bench line, then the training step's kernel stats
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_X=0" bash tools/gpu_train_kstats.sh > gpurun_out/tks/summary.txt 2>&1
cat gpurun_out/tks/summary.txt

# Round-4 evidence run: full GPU suite + smoke + bench line, then the dominant kernel's profile
# (stamps, inference kernel stats, FETCH/WRITE and SQ passes: tools/gpu_strip_prof.sh), the
# training step's kernel stats and the training strip kernels' counter passes.  Each step is
# time-limited inside its own script; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
bash tools/gpu_strip_prof.sh > gpurun_out/prof3.txt 2>&1
echo "strip prof done"; tail -30 gpurun_out/prof3.txt
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_X=0" bash tools/gpu_train_kstats.sh > gpurun_out/tks/summary.txt 2>&1
cat gpurun_out/tks/summary.txt
bash tools/gpu_train_pmc.sh > gpurun_out/tpmc.txt 2>&1
echo "train pmc done"; tail -50 gpurun_out/tpmc.txt

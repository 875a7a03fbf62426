# Round-5 evidence: the bench's inference leg under rocprofv3 --kernel-trace --stats, the dominant
# launch's FETCH_SIZE / WRITE_SIZE and SQ passes (tools/gpu_chain_prof.sh), then the stage-1
# training step's kernel stats (tools/gpu_train_kstats.sh)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_chain_prof.sh > gpurun_out/profc.txt 2>&1
echo "chain prof done"; tail -12 gpurun_out/profc.txt
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_X=0" bash tools/gpu_train_kstats.sh > gpurun_out/tks/summary.txt 2>&1
cat gpurun_out/tks/summary.txt

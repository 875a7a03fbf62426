export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_strip_prof.sh > gpurun_out/prof3.txt 2>&1; echo "strip prof rc=$?"; tail -40 gpurun_out/prof3.txt
mkdir -p gpurun_out/tks
AB_CONFIGS="FEN_X=0" bash tools/gpu_train_kstats.sh > gpurun_out/tks/summary.txt 2>&1 && cat gpurun_out/tks/summary.txt && \
bash tools/gpu_train_pmc.sh > gpurun_out/tpmc.txt 2>&1; echo "train pmc rc=$?"; tail -60 gpurun_out/tpmc.txt

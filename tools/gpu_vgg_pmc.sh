# full GPU suite + smoke + bench line on the current tree, then the VGG wide conv's
# SQ counters (c3_2 forward, 64 x 64 x 256 -> 256 at N = 64) and the perceptual step's kernel stats
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
mkdir -p gpurun_out/pmc_v
i=0
for set in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM" "SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc_v/p$i -o run --output-format csv -- python tools/pmc_vggconv.py > gpurun_out/pmc_v/log$i.txt 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/pmc_v/log$i.txt; exit 1; }
done
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_v/kt -o run --output-format csv -- python tools/pmc_vggconv.py > gpurun_out/pmc_v/logkt.txt 2>&1
PERCEPTUAL=1 STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_v/perc -o run --output-format csv -- python tools/train_step.py > gpurun_out/pmc_v/perc.log 2>&1
echo ALL_OK

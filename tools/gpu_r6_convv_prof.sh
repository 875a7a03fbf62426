# round 6: k_conv3x3_v counters on the VGG c3_2 shape (fwd, dgrad) + the perceptual step's kernel
# breakdown with the wide conv on / off
export TMPDIR=/tmp
mkdir -p gpurun_out/convvp
i=0
for dg in 0 1; do
for set in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM"; do
  i=$((i + 1))
  DGRAD=$dg timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/convvp/p$i -o run --output-format csv -- python tools/pmc_vggconv.py > gpurun_out/convvp/log$i.txt 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/convvp/log$i.txt; exit 1; }
done; done
for v in 0 1; do
  FEN_CONV_V=$v PERCEPTUAL=1 STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/convvp/perc$v -o run --output-format csv -- python tools/train_step.py > gpurun_out/convvp/perc$v.log 2>&1 || exit 1
done

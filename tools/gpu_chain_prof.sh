# fen_group_strip_chain evidence pass (the bench's dominant launch since round 4): the bench under
# rocprofv3 kernel-trace --stats, FETCH_SIZE / WRITE_SIZE and SQ counter passes on tools/pmc_strip.py
# CHAIN=6 (the body's 6 groups in one launch)
export CHAIN=6 REPS=6
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/profc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profc/inf -o run --output-format csv -- \
    python bench.py --no-train --no-stress --no-cpu-baseline > gpurun_out/profc/inf_bench.log 2>&1
echo "inf rc=$?"
python tools/prof_summary.py stats "$(find gpurun_out/profc/inf -name '*kernel_stats.csv' | head -1)" gpurun_out/profc/inference_kernel_stats.csv
head -8 gpurun_out/profc/inference_kernel_stats.csv
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/profc/fetch -o run --output-format csv -- python tools/pmc_strip.py > gpurun_out/profc/fetch.log 2>&1
echo "fetch rc=$?"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/profc/write -o run --output-format csv -- python tools/pmc_strip.py > gpurun_out/profc/write.log 2>&1
echo "write rc=$?"
ALG=$(grep algorithmic_bytes_per_launch gpurun_out/profc/fetch.log | awk '{print $2}')
python tools/prof_summary.py pmc "$(find gpurun_out/profc/fetch -name '*counter_collection.csv' | head -1)" \
    "$(find gpurun_out/profc/write -name '*counter_collection.csv' | head -1)" gpurun_out/profc/pmc_k_group_strip_chain.json \
    "k_group_strip chain" "$ALG" "k_group_strip chain (the body: 6 ResidualGroups x (10 RCABs + group conv) + conv_after_body, one launch), fp16, B=32, 64x64x64" "k_group_strip!bwd"
cat gpurun_out/profc/pmc_k_group_strip_chain.json
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/profc/sq$i -o run --output-format csv -- python tools/pmc_strip.py > gpurun_out/profc/sq$i.log 2>&1 || { echo "pass $i failed"; continue; }
  f=$(find gpurun_out/profc/sq$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_group_strip' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    v = v[1:] or v
    print(f"{k:32s} {sum(v) / len(v):16.0f}")
PY
done <<'SETS' > gpurun_out/profc/sq_counters.txt 2>&1
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CU_CYCLES
SETS
cat gpurun_out/profc/sq_counters.txt

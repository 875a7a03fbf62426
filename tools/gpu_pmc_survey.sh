# Counter survey of the dominant kernel (tools/pmc_rcab.py): the available counter list, then
# SQ pass(es) of wait / busy / instruction-mix counters, each pass its own run.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcs
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcs/list.txt 2>&1 || true
grep -oE "\bSQ_[A-Z0-9_]+\b|\bTA_[A-Z0-9_]+\b|\bTD_[A-Z0-9_]+\b|\bTCP_[A-Z0-9_]+\b" gpurun_out/pmcs/list.txt | sort -u > gpurun_out/pmcs/names.txt || true
wc -l gpurun_out/pmcs/names.txt
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set -d gpurun_out/pmcs/p$i -o run --output-format csv -- python tools/pmc_rcab.py > gpurun_out/pmcs/p$i.log 2>&1 || { echo "pass $i failed: $set"; continue; }
  f=$(find gpurun_out/pmcs/p$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_rcab' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    v = v[2:] or v
    print(f"{k:32s} {sum(v) / len(v):16.0f}")
PY
done <<'SETS'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CU_CYCLES
SETS

# SQ counter passes on the 128-channel kernel (tools/pmc_c128.py), one pass per counter set,
# averaged per mode (kernel name) over the launches after the first two repetitions
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/c128pmc
mkdir -p $D
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $D/sq$i -o run --output-format csv -- python tools/pmc_c128.py > $D/sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  f=$(find $D/sq$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get('Kernel_Name', '')
    if 'k_rcab128' in n:
        mode = n.split('k_rcab128')[1][:14]
        agg[(mode, r['Counter_Name'])].append(float(r['Counter_Value']))
for (mode, k), v in sorted(agg.items()):
    v = v[len(v) // 5:] or v
    print(f"{mode:16s} {k:28s} {sum(v) / len(v):16.0f}")
PY
done <<'SETS' > $D/sq_counters.txt 2>&1
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CU_CYCLES
SETS
cat $D/sq_counters.txt

# SQ counter passes of the batched weight-gradient kernel (k_wgrad_p<64>) in eager stage-1 steps
# (tools/pmc_train.py); per-launch averages after the first two steps
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/wgpmc
mkdir -p $D
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $D/sq$i -o run --output-format csv -- python tools/pmc_train.py > $D/sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  f=$(find $D/sq$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get('Kernel_Name', '')
    if 'k_wgrad_p<64>' in n or 'k_wgrad_pILi64' in n:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    v = v[len(v) // 3:] or v
    print(f"k_wgrad_p<64> {k:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
PY
done <<'SETS' > $D/sq_counters.txt 2>&1
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CU_CYCLES
SETS
cat $D/sq_counters.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python tools/pmc_train.py > $D/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- python tools/pmc_train.py > $D/write.log 2>&1
python tools/prof_summary.py pmc "$(find $D/fetch -name '*counter_collection.csv' | head -1)" "$(find $D/write -name '*counter_collection.csv' | head -1)" $D/pmc_wgrad.json "k_wgrad_p<64>" 282329088 "k_wgrad_p<64>, 8 jobs of 64->64 at B=32 64x64 (x, dy 16.8 MB each per job)"

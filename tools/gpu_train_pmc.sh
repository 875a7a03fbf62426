# Training strip kernels' counter passes (tools/pmc_train.py, eager stage-1 steps): FETCH_SIZE and
# WRITE_SIZE (separate passes) -> HBM bytes per launch against the algorithmic bytes, then SQ sets
# for k_group_strip (training form) and k_group_strip_bwd.  Output under gpurun_out/tpmc/.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/tpmc
mkdir -p $D
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python tools/pmc_train.py > $D/fetch.log 2>&1
echo "fetch ok"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- python tools/pmc_train.py > $D/write.log 2>&1
echo "write ok"
FC=$(find $D/fetch -name '*counter_collection.csv' | head -1)
WC=$(find $D/write -name '*counter_collection.csv' | head -1)
AF=$(grep algorithmic_bytes_fwd_train $D/fetch.log | awk '{print $2}')
AB=$(grep algorithmic_bytes_bwd $D/fetch.log | awk '{print $2}')
python tools/prof_summary.py pmc "$FC" "$WC" $D/pmc_k_group_strip_train.json "k_group_strip!bwd" "$AF" \
    "k_group_strip, training form (a ResidualGroup's forward + the backward's operands), bf16, B=32, 64x64x64"
python tools/prof_summary.py pmc "$FC" "$WC" $D/pmc_k_group_strip_bwd.json "k_group_strip_bwd" "$AB" \
    "k_group_strip_bwd (a ResidualGroup's backward data gradients + SE backward), bf16, B=32, 64x64x64"
i=0
while read -r set; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $D/sq$i -o run --output-format csv -- python tools/pmc_train.py > $D/sq$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  f=$(find $D/sq$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
for key in ("k_group_strip!bwd", "k_group_strip_bwd"):
    sub, _, excl = key.partition("!")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        n = r.get('Kernel_Name', '')
        if sub in n and not (excl and excl in n):
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in sorted(agg.items()):
        v = v[12:] or v      # drop the first two steps' launches (6 groups per step)
        print(f"{key:20s} {k:32s} {sum(v) / len(v):16.0f}")
PY
done <<'SETS' > $D/sq_counters.txt 2>&1
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CU_CYCLES
SETS
cat $D/sq_counters.txt

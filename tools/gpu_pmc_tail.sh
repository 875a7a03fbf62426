# SQ counter passes over the stage-1 training step's launches (tools/op_times.py, TRAIN=1, each
# launch replayed REPS times), aggregated per kernel: the tail convs (k_conv3x3_g upsampler,
# k_conv3x3_s upsampler dgrads, k_cl_bwd), the batched wgrads and the strip kernels.  Each
# pass its own run, <= 8 SQ counters.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmct
i=0
while read -r set; do
  i=$((i+1))
  REPS=3 TRAIN=1 timeout -s KILL 240 rocprofv3 --pmc $set -d gpurun_out/pmct/p$i -o run --output-format csv -- python tools/op_times.py > gpurun_out/pmct/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc: $set"; tail -3 gpurun_out/pmct/p$i.log; exit 1; }
  f=$(find gpurun_out/pmct/p$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get('Kernel_Name', '')
    for key in ('k_conv3x3_g', 'k_conv3x3_s', 'k_cl_bwd', 'k_wgrad_p', 'k_group_strip_bwd', 'k_group_strip<', 'k_conv_last<'):
        if key in n:
            agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in sorted(agg.items()):
    for c, v in sorted(d.items()):
        print(f"{k:20s} {c:28s} {sum(v) / len(v):16.0f} (n={len(v)})")
PY
done <<'SETS'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM
SETS

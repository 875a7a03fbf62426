# round-5 batch p: SQ counter passes of fen_ssim_ex's two kernels (MODE=ex), per kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/ssimp
i=0
while read -r set; do
  i=$((i+1))
  MODE=ex REPS=10 timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/ssimp/sq$i -o run --output-format csv -- python tools/ssim_run.py > gpurun_out/ssimp/sq$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -3 gpurun_out/ssimp/sq$i.log; exit 1; }
  f=$(find gpurun_out/ssimp/sq$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get('Kernel_Name', '')
    if 'k_ssim' in n:
        k = 'g2' if 'g2' in n else 'map'
        agg[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    v = v[3:] or v
    print(f"{k[0]:4s} {k[1]:32s} {sum(v) / len(v):16.0f}")
PY
done <<'SETS' > gpurun_out/ssimp/sq_counters.txt 2>&1
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC
SETS
cat gpurun_out/ssimp/sq_counters.txt

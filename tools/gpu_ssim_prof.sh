# k_ssim<GRAD> evidence: timing of the product and build_var variants, then SQ counter passes
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ssim
for l in face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null); do
  echo "$(basename $l): $(FEN_HIP_LIB=$l timeout -k 10 100 python tools/ssim_run.py 2>&1 | tail -1)"
done
[ "${PMC:-1}" = "1" ] || exit 0
i=0
while read -r set; do
  i=$((i+1))
  REPS=10 timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/ssim/sq$i -o run --output-format csv -- python tools/ssim_run.py > gpurun_out/ssim/sq$i.log 2>&1 || { echo "pass $i failed"; continue; }
  f=$(find gpurun_out/ssim/sq$i -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_ssim' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    v = v[3:] or v
    print(f"{k:32s} {sum(v) / len(v):16.0f}")
PY
done <<'SETS' > gpurun_out/ssim/sq_counters.txt 2>&1
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC
SETS
cat gpurun_out/ssim/sq_counters.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ssim/fetch -o run --output-format csv -- python tools/ssim_run.py > gpurun_out/ssim/fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ssim/write -o run --output-format csv -- python tools/ssim_run.py > gpurun_out/ssim/write.log 2>&1 && \
python tools/prof_summary.py pmc "$(find gpurun_out/ssim/fetch -name '*counter_collection.csv' | head -1)" \
    "$(find gpurun_out/ssim/write -name '*counter_collection.csv' | head -1)" gpurun_out/ssim/pmc_k_ssim.json \
    "k_ssim" 186646528 "k_ssim<GRAD> (stage-2 SSIM map + tile sums + gradient into NHWC16 bf16 dL/dsr), B=32, 3x256x256"

# LDS / MFMA counters of the fused RCAB (one --pmc pass, SQ block only)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_lds
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc_lds -o run --output-format csv -- python tools/pmc_rcab.py > gpurun_out/pmc_lds/log.txt 2>&1
f=$(find gpurun_out/pmc_lds -name '*counter_collection.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if 'k_rcab' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    print(k, len(v), sum(v) / len(v))
PY

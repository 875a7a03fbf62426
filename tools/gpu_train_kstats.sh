# Per-kernel averages of the training step under each configuration of $AB_CONFIGS
# (';'-separated VAR=value lists): rocprofv3 --kernel-trace --stats of tools/train_step.py.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra CFGS <<< "${AB_CONFIGS:-FEN_SE_BWD=pair;FEN_SE_BWD=fused}"
i=0
for v in "${CFGS[@]}"; do
  i=$((i + 1))
  env $v STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tks/c$i -o run --output-format csv -- python tools/train_step.py > gpurun_out/tks/c$i.log 2>&1
  f=$(find gpurun_out/tks/c$i -name '*kernel_stats.csv' | head -1)
  echo "== $v"
  python - "$f" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:14]:
    print(f"{float(x['TotalDurationNs'])/1e6:8.2f} ms {int(x['Calls']):6d} {float(x['AverageNs'])/1e3:7.1f} us  {x['Name'][:80]}")
PY
done

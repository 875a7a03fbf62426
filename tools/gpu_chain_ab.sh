# Same-box A/B of the chained body launch (FEN_GROUP_CHAIN=1) against a launch per group (=0):
# per-launch times (tools/op_times.py) and the inference bench leg, interleaved x2
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chainab
for rep in 1 2; do
  for v in 1 0; do
    FEN_GROUP_CHAIN=$v timeout -k 10 200 python tools/op_times.py > gpurun_out/chainab/op_${v}_$rep.txt 2>&1 || { echo "op_times $v failed"; exit 1; }
    echo "chain=$v r$rep: $(grep -E 'group_strip' gpurun_out/chainab/op_${v}_$rep.txt | head -2 | tr -s ' ' | tr '\n' '|') $(grep 'sum of launches' gpurun_out/chainab/op_${v}_$rep.txt)"
    FEN_GROUP_CHAIN=$v timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 40 --warmup 5 > gpurun_out/chainab/b.json 2> gpurun_out/chainab/b.log || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/chainab/b.json').read().strip().splitlines()[-1]); print('   bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['bf16']['value'])"
  done
done

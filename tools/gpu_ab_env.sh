# Same-box A/B of an environment switch on the inference bench: runs `bench.py --no-train
# --no-stress --no-cpu-baseline` alternately with $AB_OFF and $AB_ON (e.g. AB_OFF=FEN_RCAB_REV=0
# AB_ON=FEN_RCAB_REV=1), $REPS times each; prints value / ms per step / dominant-kernel us.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abenv
for r in $(seq 1 ${REPS:-2}); do
  for v in "$AB_OFF" "$AB_ON"; do
    env $v timeout -k 10 300 python bench.py --no-train --no-stress --no-cpu-baseline --steps ${STEPS:-100} > gpurun_out/abenv/b.json 2> gpurun_out/abenv/b.log
    python -c "import json; d=json.loads(open('gpurun_out/abenv/b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], 'bf16', d['bf16']['value'], d['bf16']['ms_per_step'])"
  done
done

# fen_group_strip_bwd: parity tests (vs the oracle's autograd and the per-RCAB backward, graph
# replay), then the stage-1 training leg with the strip backward on / off (same box)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_group_strip_bwd.py -m gpu -v -s -x --timeout 300 --timeout-method thread > gpurun_out/sb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|error|dx strip|worst|assert" gpurun_out/sb_tests.log | tail -40
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in 1 0; do
    FEN_GROUP_STRIP_BWD=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-stress --no-perceptual --steps 10 --warmup 3 --train-steps 20 > gpurun_out/sbt_$v.json 2> gpurun_out/sbt_$v.log
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/sbt_$v.log; exit $rc; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/sbt_{sys.argv[1]}.json").read().strip().splitlines()[-1])
t = d["train"]
print(f"strip_bwd={sys.argv[1]}  inference {d['value']:9.1f} img/s  train {t['ms_per_step']:7.3f} ms  loss {t['loss']:.6f}  gan {d.get('train_gan', {}).get('ms_per_step')}")
PY
  done
done

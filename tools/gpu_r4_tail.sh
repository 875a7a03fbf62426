# FEN_TAIL_CHUNK A/B: the tail-chunk parity tests, then the inference bench leg at chunk 0 / 16 / 8 / 4
# (two alternating rounds) and the per-launch times at chunk 8.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tail
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_gpu_northstar.py::test_g9_engine_tail_chunks tests/test_gpu_rcab128.py::test_rcab128_net_tail_chunks \
    > gpurun_out/tail/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|dPSNR" gpurun_out/tail/tests.log | tail -8
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for c in 0 16 8 4; do
    FEN_TAIL_CHUNK=$c timeout -k 10 200 python bench.py --no-train --no-stress --no-cpu-baseline \
        > gpurun_out/tail/b_${c}_$r.json 2> gpurun_out/tail/b_${c}_$r.log || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/tail/b_${c}_$r.json "chunk=$c r$r"
  done
done
FEN_TAIL_CHUNK=8 timeout -k 10 200 python tools/op_times.py > gpurun_out/tail/op8.txt 2>&1
echo "op8 rc=$?"; tail -14 gpurun_out/tail/op8.txt

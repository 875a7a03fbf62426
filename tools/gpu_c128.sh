# fen_rcab_c128: parity tests, then the stress leg (configs[4]) with the fused launches on / off
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rcab128.py -m gpu -v -s -x --timeout 300 --timeout-method thread > gpurun_out/c128_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|error|rel |assert" gpurun_out/c128_tests.log | tail -40
[ $rc -eq 0 ] || exit 1
for v in 1 0; do
  FEN_RCAB_C128=$v STEPS=5 timeout -k 10 300 python tools/stress_step.py > gpurun_out/c128_stress_$v.log 2>&1 || { echo "stress rc=$?"; tail -5 gpurun_out/c128_stress_$v.log; exit 1; }
  echo "c128=$v $(tail -1 gpurun_out/c128_stress_$v.log)"
done

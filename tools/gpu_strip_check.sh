# fen_group_strip: parity tests, then the inference bench legs (fp16 / bf16) and a kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_strip.py -m gpu -v -s -x --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1
rc=$?; echo "strip tests rc=$rc"; grep -E "rel |PASS|FAIL|passed|failed|Error" gpurun_out/gs_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 250 python -u -m pytest tests/test_gpu_train64.py tests/test_gpu_rcab.py -m gpu -v -s --timeout 200 --timeout-method thread -k "train64 or se_fold_vs_oracle" > gpurun_out/t64.log 2>&1
rc=$?; echo "train64 rc=$rc"; grep -E "worst|PASS|FAIL|passed|failed" gpurun_out/t64.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-train --no-cpu-baseline --no-stress --steps 30 --warmup 5 > gpurun_out/bench_strip.json 2> gpurun_out/bench_strip.log
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_strip.json

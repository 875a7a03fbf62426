# fen_group_strip: parity tests, phase stamps (diagnostic library), the inference bench legs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_strip.py -m gpu -v -s -x --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1
rc=$?; echo "strip tests rc=$rc"; grep -E "rel |PASS|FAIL|passed|failed|Error" gpurun_out/gs_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip.py > gpurun_out/stamps.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/stamps.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-train --no-cpu-baseline --no-stress --steps 30 --warmup 5 > gpurun_out/bench_strip.json 2> gpurun_out/bench_strip.log
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_strip.json | cut -c1-900

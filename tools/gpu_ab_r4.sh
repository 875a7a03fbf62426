# round-4 A/B: parity tests of the strip kernels, then the inference bench leg and the stage-1
# training step for the product library and every variant in csrc/build_var, interleaved x2;
# then (DPOV=1) the DP exchange overlap measurement
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_group_strip.py tests/test_gpu_group_strip_bwd.py tests/test_gpu_strip_status.py tests/test_gpu_ssim.py} -m gpu -v -s -x --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/ab_tests.log | tail -4
[ $rc -eq 0 ] || { tail -30 gpurun_out/ab_tests.log; exit 1; }
libs="face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null)"
for rep in 1 2; do
  for l in $libs; do
    FEN_HIP_LIB=$l timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 30 --warmup 5 > gpurun_out/ab_b.json 2> gpurun_out/ab_b.log
    rc=$?; [ $rc -eq 0 ] || { echo "bench $l rc=$rc"; tail -5 gpurun_out/ab_b.log; exit $rc; }
    python - "$l" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_b.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1].split('/')[-1]:28s} {d['value']:9.1f} img/s  kernel {r['kernel_ms']*1e3:7.1f} us  frac {r['frac']:.4f}  bf16 {d['bf16']['value']:9.1f} ({d['bf16']['kernel_ms']*1e3:.1f} us)")
PY
    FEN_HIP_LIB=$l STEPS=20 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "   $(tail -1 gpurun_out/ab_t.log)"
  done
done
timeout -k 10 120 python tools/bench_ssim.py 2>&1 | grep -v amdgpu.ids | tail -3
timeout -k 10 120 python tools/op_times.py 2>&1 | grep -v amdgpu.ids | tail -30
[ "${TRAINOPS:-0}" = "1" ] && { TRAIN=1 timeout -k 10 300 python tools/op_times.py 2>&1 | grep -v amdgpu.ids | tail -60; }
if [ "${STAMPS:-0}" = "1" ] && [ -f face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so ]; then
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip.py 2>&1 | grep -v amdgpu.ids
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip_bwd.py 2>&1 | grep -v amdgpu.ids
fi
if [ "${UPSTAMP:-0}" = "1" ]; then
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so UP=1 REPS=12000 timeout -k 10 200 python tools/stamp_conv.py 2>&1 | grep -v amdgpu.ids
fi
if [ "${DPOV:-0}" = "1" ]; then
  timeout -k 10 400 python tools/dp_overlap.py > gpurun_out/dp_overlap.json 2> gpurun_out/dp_overlap.log
  rc=$?; grep -v amdgpu.ids gpurun_out/dp_overlap.log | tail -8; cat gpurun_out/dp_overlap.json; exit $rc
fi

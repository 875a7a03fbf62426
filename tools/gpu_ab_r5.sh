# round-5 A/B: parity tests (TESTS), then the stage-1 training step (and, INF=1, the inference
# bench leg) for the product library and every variant in csrc/build_var, interleaved x REPS;
# STAMPS=1: the strip kernels' stamp timelines from build_stamp
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v -s -x --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/ab_tests.log | tail -4
  [ $rc -eq 0 ] || { tail -40 gpurun_out/ab_tests.log; exit 1; }
fi
libs="face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null)"
for rep in $(seq 1 ${REPS:-2}); do
  for l in $libs; do
    if [ "${INF:-0}" = "1" ]; then
      FEN_HIP_LIB=$l timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 30 --warmup 5 > gpurun_out/ab_b.json 2> gpurun_out/ab_b.log
      rc=$?; [ $rc -eq 0 ] || { echo "bench $l rc=$rc"; tail -5 gpurun_out/ab_b.log; exit $rc; }
      python - "$l" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_b.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1].split('/')[-1]:28s} {d['value']:9.1f} img/s  kernel {r['kernel_ms']*1e3:7.1f} us  frac {r['frac']:.4f}  bf16 {d['bf16']['value']:9.1f} ({d['bf16']['kernel_ms']*1e3:.1f} us)")
PY
    fi
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done
if [ "${STAMPS:-0}" = "1" ] && [ -f face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so ]; then
  FEN_GROUP_CHAIN=0 FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip_bwd.py 2>&1 | grep -v amdgpu.ids
fi

# fen_group_strip A/B: parity tests on the product library, then the inference bench leg for the
# product library and every variant in csrc/build_var (make variant V=... DEFS=...), twice each
# interleaved, then the stamp table of the diagnostic build
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_strip.py -m gpu -v -s -x --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1
rc=$?; echo "strip tests rc=$rc"; grep -E "rel |passed|failed|Error" gpurun_out/gs_tests.log | tail -8
[ $rc -eq 0 ] || exit 1
libs="face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null)"
for rep in 1 2; do
  for l in $libs; do
    FEN_HIP_LIB=$l timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 30 --warmup 5 > gpurun_out/ab_b.json 2> gpurun_out/ab_b.log
    rc=$?; [ $rc -eq 0 ] || { echo "bench $l rc=$rc"; tail -5 gpurun_out/ab_b.log; exit $rc; }
    python - "$l" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_b.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1].split('/')[-1]:32s} {d['value']:9.1f} img/s  kernel {r['kernel_ms']*1e3:7.1f} us  frac {r['frac']:.4f}  bf16 {d['bf16']['value']:9.1f}")
PY
  done
done
if [ -f face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so ]; then
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip.py > gpurun_out/stamps.txt 2>&1
  rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.txt
fi

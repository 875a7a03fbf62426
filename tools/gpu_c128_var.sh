# 128-channel kernel variants (csrc/build_var/libfen_hip_*.so): parity tests on each variant, then
# the stress leg A/B (product vs variants, 2 reps interleaved) and the variants' kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
for l in face-super-resolution_amd/csrc/build_var/libfen_hip_*.so; do
  FEN_HIP_LIB=$l timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab128.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c128var_tests.log 2>&1
  rc=$?; echo "$(basename $l) tests rc=$rc: $(tail -1 gpurun_out/c128var_tests.log)"; [ $rc -eq 0 ] || exit 1
done
for rep in 1 2; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_*.so; do
    FEN_HIP_LIB=$l STEPS=5 timeout -k 10 300 python tools/stress_step.py > gpurun_out/c128_ab.log 2>&1 || { echo "stress rc=$?"; tail -5 gpurun_out/c128_ab.log; exit 1; }
    echo "$(basename $l) $(tail -1 gpurun_out/c128_ab.log | python -c 'import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms", d["frac_peak"])')"
  done
done
for l in face-super-resolution_amd/csrc/build_var/libfen_hip_*.so; do
  FEN_HIP_LIB=$l STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c128var/p -o run --output-format csv -- python tools/stress_step.py > gpurun_out/c128var.log 2>&1 || exit 1
  python tools/prof_summary.py stats "$(find gpurun_out/c128var/p -name '*kernel_stats.csv' | head -1)" gpurun_out/c128var_stats.csv | head -6
done

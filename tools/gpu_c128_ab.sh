# fen_rcab_c128: parity tests on the product library, then the stress leg (configs[4]) A/B against
# a variant library ($VAR, default build_var/libfen_hip_r128v1.so) on one box, then rocprofv3 stats
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=${VAR:-face-super-resolution_amd/csrc/build_var/libfen_hip_r128v1.so}
timeout -k 10 600 python -u -m pytest tests/test_gpu_rcab128.py -m gpu -v -s -x --timeout 300 --timeout-method thread > gpurun_out/c128_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|error|rel |assert|max " gpurun_out/c128_tests.log | tail -30
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for lib in "$VAR" face-super-resolution_amd/src/hip/libfen_hip.so; do
    FEN_HIP_LIB=$lib STEPS=5 timeout -k 10 300 python tools/stress_step.py > gpurun_out/c128_ab.log 2>&1 || { echo "stress rc=$?"; tail -5 gpurun_out/c128_ab.log; exit 1; }
    echo "$(basename $lib) $(tail -1 gpurun_out/c128_ab.log | python -c 'import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms", d["frac_peak"])')"
  done
done
bash tools/gpu_stress_prof.sh

# k_ssim<GRAD>: the SSIM GPU tests on the product library, then timing of the product and the
# build_var variants (tools/ssim_run.py), interleaved x2
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ssim
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_bench_legs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ssim/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ssim/tests.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for l in face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null); do
  echo "$(basename $l): $(FEN_HIP_LIB=$l timeout -k 10 100 python tools/ssim_run.py 2>&1 | tail -1)"
done
done

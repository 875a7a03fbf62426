set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1
for v in apf xpre; do
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1
done
timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1

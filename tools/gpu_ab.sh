# A/B: bench_rcab on the product library and on each build_var/ variant given as arguments
set -e
export TMPDIR=/tmp
echo "default $(timeout -k 10 120 python tools/bench_rcab.py 2>&1 | tail -1)"
for v in "$@"; do
  echo "$v $(FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 120 python tools/bench_rcab.py 2>&1 | tail -1)"
done

set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 python tools/bench_last.py
for v in nocomp noload; do
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 60 python tools/bench_last.py
done

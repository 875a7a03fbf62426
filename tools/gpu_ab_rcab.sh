# A/B of k_rcab builds on one box: default library vs build_var variants named in $VARIANTS
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  echo -n "default "; timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1
  for v in ${VARIANTS:-nont}; do
    echo -n "$v "; FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so timeout -k 10 120 python -u tools/bench_rcab.py 2>&1 | tail -1
  done
done

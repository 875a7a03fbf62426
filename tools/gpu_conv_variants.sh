# conv kernel variants: microbench (graph-replayed), ablations, phase stamps, MFMA loop
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 3 4; do
  FEN_CONV_VARIANT=$v ABLATE=1 timeout -k 10 120 python tools/bench_conv.py
done
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so timeout -k 10 120 python tools/stamp_conv.py
FEN_CONV_VARIANT=4 FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so timeout -k 10 120 python tools/stamp_conv.py
timeout -k 10 60 tools/mfma_loop

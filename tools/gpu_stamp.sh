set -e
export FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so
for b in 32 128; do
  B=$b timeout -k 10 120 python tools/stamp_conv.py
done
B=32 EPI=0 timeout -k 10 120 python tools/stamp_conv.py

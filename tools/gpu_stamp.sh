set -e
export FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so
B=32 FEN_CONV_VARIANT=4 timeout -k 10 120 python tools/stamp_conv.py
B=32 timeout -k 10 120 python tools/stamp_conv.py

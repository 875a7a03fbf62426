set -e
export TMPDIR=/tmp
L=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so
FEN_HIP_LIB=$L timeout -k 10 120 python tools/stamp_conv.py
FEN_HIP_LIB=$L EPI=32 timeout -k 10 120 python tools/stamp_conv.py
FEN_HIP_LIB=$L FEN_CONV_VARIANT=5 timeout -k 10 120 python tools/stamp_conv.py

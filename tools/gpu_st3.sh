set -e
export TMPDIR=/tmp
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so timeout -k 10 120 python -u tools/stamp_rcab.py

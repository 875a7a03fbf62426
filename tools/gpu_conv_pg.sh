# ping-pong (variant 0) vs persistent (variant 5) conv kernel per epilogue mode
set -e
export TMPDIR=/tmp
for v in 0 5; do
  FEN_CONV_VARIANT=$v timeout -k 10 120 python tools/bench_conv.py | head -1
done

export TMPDIR=/tmp
for rep in 1 2; do for v in prod nowait nobar nodma nomma; do
  if [ $v = prod ]; then L=face-super-resolution_amd/src/hip/libfen_hip.so; else L=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so; fi
  FEN_HIP_LIB=$L timeout -k 10 120 python tools/bench_vgg_conv.py > gpurun_out/ab_v.txt 2>&1 || { tail -3 gpurun_out/ab_v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_v.txt)"
done; done
FEN_CONV_V=0 timeout -k 10 120 python tools/bench_vgg_conv.py > gpurun_out/ab_v.txt 2>&1 && echo "streamed $(tail -1 gpurun_out/ab_v.txt)"

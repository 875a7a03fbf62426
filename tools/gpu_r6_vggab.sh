# bench_vgg_conv over library variants (VARIANTS; "prod" = the product library), REPS reps
export TMPDIR=/tmp
mkdir -p gpurun_out/vab
V=face-super-resolution_amd/csrc/build_var
for rep in $(seq 1 ${REPS:-2}); do
  for l in prod $VARIANTS; do
    if [ $l = prod ]; then L=face-super-resolution_amd/src/hip/libfen_hip.so; else L=$V/libfen_hip_$l.so; fi
    FEN_HIP_LIB=$L timeout -k 10 120 python tools/bench_vgg_conv.py > gpurun_out/vab/vgg.txt 2>&1 || { tail -3 gpurun_out/vab/vgg.txt; exit 1; }
    echo "$l $(tail -1 gpurun_out/vab/vgg.txt)"
  done
done

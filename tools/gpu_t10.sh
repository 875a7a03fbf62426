set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
true

for v in new pre new pre; do
  if [ $v = pre ]; then export FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_pre.so; else unset FEN_HIP_LIB; fi
  timeout -k 10 200 python bench.py --no-train --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
unset FEN_HIP_LIB
timeout -k 10 120 python tools/bench_conv.py
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_pre.so timeout -k 10 120 python tools/bench_conv.py

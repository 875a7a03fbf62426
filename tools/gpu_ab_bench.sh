set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new old new old; do
  if [ $v = old ]; then export FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_old.so; else unset FEN_HIP_LIB; fi
  timeout -k 10 200 python bench.py --no-train --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done

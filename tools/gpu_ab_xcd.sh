# A/B of the XCD-aware block mapping: default library vs variants without it (conv kernels only / all)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new convnoxcd noxcd new convnoxcd noxcd; do
  if [ $v = new ]; then unset FEN_HIP_LIB; else export FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so; fi
  timeout -k 10 200 python bench.py --no-perceptual --no-stress --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['train']['value'], d['train']['ms_per_step'])"
done

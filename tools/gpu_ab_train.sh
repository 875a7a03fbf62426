# A/B of library variants (build_var/libfen_hip_$v.so, names in $VARIANTS) against the default
# library on the inference step and the stage-1 training step
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in new ${VARIANTS}; do
    if [ $v = new ]; then unset FEN_HIP_LIB; else export FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$v.so; fi
    timeout -k 10 200 python bench.py --no-perceptual --no-stress --no-cpu-baseline --steps 20 --train-steps 20 > gpurun_out/ab_$v.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_ms'], d['train']['value'], d['train']['ms_per_step'])"
  done
done

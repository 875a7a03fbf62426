set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_gan_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t8.log 2>&1 || { tail -40 gpurun_out/t8.log; exit 1; }
tail -1 gpurun_out/t8.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/t8_bench.log 2>&1
tail -1 gpurun_out/t8_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['train']['ms_per_step'], d['train_perceptual']['ms_per_step'], d['train_gan']['ms_per_step'])"

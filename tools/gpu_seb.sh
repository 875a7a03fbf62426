# the SE backward folded into the fused RCAB backward: parity (fold vs two launches, the RCAB /
# net / module / perceptual / GAN tests), then same-box A/B of FEN_SE_IN_BWD on the train step
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_seb.log 2>&1 || { tail -40 gpurun_out/pytest_seb.log; exit 1; }
tail -2 gpurun_out/pytest_seb.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_perceptual_train.py tests/test_gpu_gan_step.py tests/test_gpu_lite.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_seb2.log 2>&1 || { tail -40 gpurun_out/pytest_seb2.log; exit 1; }
tail -2 gpurun_out/pytest_seb2.log
for r in 1 2; do
  for v in FEN_SE_IN_BWD=launch FEN_SE_IN_BWD=fold; do
    echo "$v | $(env $v STEPS=30 timeout -k 10 300 python tools/train_step.py 2>/dev/null | tail -1)"
  done
done

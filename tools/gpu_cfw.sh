set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k conv_first -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_cfw.log 2>&1 || { tail -40 gpurun_out/pytest_cfw.log; exit 1; }
tail -2 gpurun_out/pytest_cfw.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_disc.py tests/test_gpu_gan_step.py tests/test_gpu_lite.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cfw2.log 2>&1 || { tail -40 gpurun_out/pytest_cfw2.log; exit 1; }
tail -2 gpurun_out/pytest_cfw2.log
for r in 1 2; do
  for v in FEN_CFW_VALU=1 FEN_X=0; do echo "$v | $(env $v timeout -k 10 300 python tools/gan_step.py | tail -1)"; done
done

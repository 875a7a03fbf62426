set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rccl.log 2>&1 || { tail -30 gpurun_out/pytest_rccl.log; exit 1; }
tail -2 gpurun_out/pytest_rccl.log
bash tools/gpu_gan_prof.sh

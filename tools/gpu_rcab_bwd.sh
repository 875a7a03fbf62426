# fused RCAB backward: kernel test, training-parity tests, same-box A/B of the training step
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py -k rcab_bwd -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rb.log 2>&1 || { tail -40 gpurun_out/pytest_rb.log; exit 1; }
tail -2 gpurun_out/pytest_rb.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_module.py tests/test_gpu_dp_engine.py tests/test_gpu_rccl.py tests/test_gpu_perceptual_train.py tests/test_gpu_trainer_resume.py tests/test_gpu_gan_step.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_rb2.log 2>&1 || { tail -40 gpurun_out/pytest_rb2.log; exit 1; }
tail -2 gpurun_out/pytest_rb2.log
AB_CONFIGS="FEN_RCAB_BWD=pair;FEN_RCAB_BWD=fused" REPS=3 bash tools/gpu_ab_train_env.sh

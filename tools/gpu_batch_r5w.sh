# round-5 batch w: the strip-backward groups' column sums on a side stream beside the batched
# weight gradients (FEN_CS_SIDE=1, the default) vs in line (FEN_CS_SIDE=0): the training-engine
# tests (north-star step, DP engine, direct RCCL captures, trainer resume, bench legs), then the
# stage-1 training step A/B (4 reps, interleaved)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train64.py tests/test_gpu_dp_engine.py tests/test_gpu_rccl.py tests/test_gpu_trainer_resume.py tests/test_gpu_perceptual_train.py tests/test_gpu_northstar.py > gpurun_out/t_w.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/t_w.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/t_w.log | head -8; exit $rc; }
for rep in 1 2 3 4; do
  for v in 1 0; do
    FEN_CS_SIDE=$v STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train side=$v rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "FEN_CS_SIDE=$v   $(tail -1 gpurun_out/ab_t.log)"
  done
done

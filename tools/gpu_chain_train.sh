# The chained body launch in training: parity tests, then the stage-1 step with a chained training
# forward (FEN_GROUP_CHAIN_TRAIN=1) against a launch per group (=0), interleaved x2
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chaint
timeout -k 10 600 python -u -m pytest tests/test_gpu_group_chain.py tests/test_gpu_train64.py tests/test_gpu_strip_status.py tests/test_gpu_group_strip_bwd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/chaint/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/chaint/tests.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in 1 0; do
    FEN_GROUP_CHAIN_TRAIN=$v STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/chaint/ts.log 2>&1 || { echo "train_step failed"; tail -5 gpurun_out/chaint/ts.log; exit 1; }
    echo "chain_train=$v r$rep: $(tail -1 gpurun_out/chaint/ts.log)"
  done
done

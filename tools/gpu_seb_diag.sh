# SEB timing diagnostics: the folded RCAB backward with its halo transform compiled out (variant libraries; results wrong, timing only) against the default
# fold and the separate launch
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcab.py -k se_fold -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sebd.log 2>&1 || { tail -40 gpurun_out/pytest_sebd.log; exit 1; }
tail -1 gpurun_out/pytest_sebd.log
VB=$GRAFT_REPO_ROOT/face-super-resolution_amd/csrc/build_var
for r in 1 2; do
  for v in FEN_SE_IN_BWD=launch FEN_SE_IN_BWD=fold FEN_HIP_LIB=$VB/libfen_hip_nohalo.so; do
    echo "$(basename $v) | $(env $v STEPS=30 timeout -k 10 300 python tools/train_step.py 2>/dev/null | tail -1)"
  done
done

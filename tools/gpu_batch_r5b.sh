# round-5 batch: parity of the product (per-strip dalpha partials in the strip backward) and of the
# gate-FC-prefetch variant (build_var/fc2e), then the inference + training A/B, 3 reps
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_strip_bwd.py tests/test_gpu_train64.py tests/test_gpu_strip_status.py tests/test_gpu_rccl.py > gpurun_out/t_prod.log 2>&1
rc=$?; echo "product tests rc=$rc"; tail -2 gpurun_out/t_prod.log; [ $rc -eq 0 ] || exit 1
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_fc2e.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_chain.py tests/test_gpu_group_strip.py > gpurun_out/t_fc2e.log 2>&1
rc=$?; echo "fc2e tests rc=$rc"; tail -2 gpurun_out/t_fc2e.log; [ $rc -eq 0 ] || exit 1
INF=1 REPS=3 bash tools/gpu_ab_r5.sh
timeout -k 10 200 python tools/op_times.py > gpurun_out/ops_inf.txt 2>&1
TRAIN=1 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train.txt 2>&1
echo "op_times rc=$?"

# round-5 A/B batch: the SE-overlapped strip backward (sev2) parity + training A/B, the gate FC
# prefetch variants (fc2e, fc12e) inference A/B, stamps of both backward forms
export TMPDIR=/tmp
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_sev2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_strip_bwd.py tests/test_gpu_train64.py tests/test_gpu_strip_status.py > gpurun_out/t_sev2.log 2>&1
echo "sev2 tests rc=$?"; tail -3 gpurun_out/t_sev2.log
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_fc2e.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_chain.py tests/test_gpu_group_strip.py > gpurun_out/t_fc2e.log 2>&1
echo "fc2e tests rc=$?"; tail -3 gpurun_out/t_fc2e.log
INF=1 REPS=3 bash tools/gpu_ab_r5.sh
FEN_GROUP_CHAIN=0 FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_sev2stamp.so timeout -k 10 200 python tools/stamp_strip_bwd_v2.py 2>&1 | grep -v amdgpu.ids
FEN_GROUP_CHAIN=0 FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip_bwd.py 2>&1 | grep -v amdgpu.ids

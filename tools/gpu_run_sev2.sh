export TMPDIR=/tmp
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_sev2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group_strip_bwd.py tests/test_gpu_train64.py tests/test_gpu_strip_status.py > gpurun_out/t_sev2.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/t_sev2.log
REPS=3 bash tools/gpu_ab_r5.sh
FEN_GROUP_CHAIN=0 FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_sev2stamp.so timeout -k 10 200 python tools/stamp_strip_bwd_v2.py 2>&1 | grep -v amdgpu.ids
FEN_GROUP_CHAIN=0 FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip_bwd.py 2>&1 | grep -v amdgpu.ids

# round-5 batch g: the 128-channel conv1's gate operands (tile sums, FC1, FC2) by LDS-DMA ahead
# of the x / t staging (product) vs through registers behind it (build_var/gatereg); the SSIM
# map kernel looping channels with prefetch.  Tests first, then the stress leg A/B, SSIM timing,
# the stress forward's per-launch trace; the training A/B against build_var/sgen (the streamed
# conv's runtime-mode epilogue)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rcab128.py tests/test_gpu_ssim.py tests/test_gpu_kernels.py tests/test_gpu_train64.py > gpurun_out/t_g.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_g.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_g.log | head -20; exit 1; }
timeout -k 10 120 python tools/bench_ssim.py > gpurun_out/ssim_g.json 2> gpurun_out/ssim_g.err
echo "bench_ssim rc=$? $(cat gpurun_out/ssim_g.json)"
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_gatereg.so; do
    FEN_HIP_LIB=$l STEPS=5 timeout -k 10 300 python tools/stress_step.py > gpurun_out/st.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "stress $l rc=$rc"; tail -5 gpurun_out/st.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/st.log)"
  done
done
for rep in 1 2 3; do
  for l in face-super-resolution_amd/src/hip/libfen_hip.so face-super-resolution_amd/csrc/build_var/libfen_hip_sgen.so; do
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/ab_t.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "train $l rc=$rc"; tail -5 gpurun_out/ab_t.log; exit $rc; }
    echo "$(echo $l | sed 's|.*/||')   $(tail -1 gpurun_out/ab_t.log)"
  done
done
TRAIN=1 REPS=10 timeout -k 10 300 python tools/op_times.py > gpurun_out/ops_train.txt 2>&1
echo "op_times rc=$?"; grep -E "conv_last|256->64|sum of" gpurun_out/ops_train.txt
# per-launch durations of the stress forward (the three upsampler stages apart)
STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/stprof -o st --output-format csv -- python tools/stress_step.py > gpurun_out/stprof.log 2>&1
echo "stress trace rc=$?"
f=$(find gpurun_out/stprof -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
last = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if ('rcab128' in n and 'Li4E' in n) or 'conv3x3_s' in n or 'conv_first' in n or ('rcab128' in n and 'Li3E' in n):
        last[n[:60]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in last.items():
    print(k, [round(x, 1) for x in v[-8:]])
PY

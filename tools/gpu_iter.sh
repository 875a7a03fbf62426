# quick iteration: kernel parity, phase stamps, conv microbench, end-to-end bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/iter_pytest.log 2>&1 || { tail -30 gpurun_out/iter_pytest.log; exit 1; }
tail -2 gpurun_out/iter_pytest.log
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so B=32 timeout -k 10 120 python tools/stamp_conv.py
FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so B=32 DEBUG=4 timeout -k 10 120 python tools/stamp_conv.py
timeout -k 10 300 python tools/bench_conv.py
timeout -k 10 300 python bench.py --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/iter_prof -o run --output-format csv -- \
    python bench.py --no-train --no-cpu-baseline --steps 20 > gpurun_out/iter_prof.log 2>&1
python tools/prof_summary.py stats gpurun_out/iter_prof/run_kernel_stats.csv gpurun_out/iter_kstats.csv

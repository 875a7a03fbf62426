# rocprofv3 passes for profiles/: kernel stats of the bench (inference, then full), and two
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) on the dominant kernel (k_rcab_d, the deferred-gate RCAB).
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/inf -o run --output-format csv -- \
    python bench.py --no-train --no-stress --no-cpu-baseline > gpurun_out/prof/inf_bench.log 2>&1
 echo INF_OK
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/full -o run --output-format csv -- \
    python bench.py --no-cpu-baseline > gpurun_out/prof/full_bench.log 2>&1
 echo FULL_OK
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- \
    python tools/pmc_rcab.py > gpurun_out/prof/fetch.log 2>&1
 echo FETCH_OK
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- \
    python tools/pmc_rcab.py > gpurun_out/prof/write.log 2>&1
 echo WRITE_OK
python tools/prof_summary.py stats "$(find gpurun_out/prof/inf -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/inference_kernel_stats.csv
python tools/prof_summary.py stats "$(find gpurun_out/prof/full -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/full_kernel_stats.csv
ALG=$(grep algorithmic_bytes_per_launch gpurun_out/prof/fetch.log | awk '{print $2}')
python tools/prof_summary.py pmc "$(find gpurun_out/prof/fetch -name '*counter_collection.csv' | head -1)" \
    "$(find gpurun_out/prof/write -name '*counter_collection.csv' | head -1)" gpurun_out/prof/pmc_k_rcab_d.json \
    k_rcab_d "$ALG" "k_rcab_d deferred-gate RCAB (inference form), fp16, B=32, 64x64x64"
tail -1 gpurun_out/prof/inf_bench.log

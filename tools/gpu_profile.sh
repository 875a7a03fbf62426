# rocprofv3 passes for profiles/: kernel stats of the bench (inference, then full), and two
# PMC passes (FETCH_SIZE, WRITE_SIZE) on the dominant kernel.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/inf -o run --output-format csv -- \
    python bench.py --no-train --no-cpu-baseline > gpurun_out/prof/inf_bench.log 2>&1 && echo INF_OK
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/full -o run --output-format csv -- \
    python bench.py --no-cpu-baseline > gpurun_out/prof/full_bench.log 2>&1 && echo FULL_OK
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- \
    python tools/pmc_rcab.py > gpurun_out/prof/fetch.log 2>&1 && echo FETCH_OK
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- \
    python tools/pmc_rcab.py > gpurun_out/prof/write.log 2>&1 && echo WRITE_OK
find gpurun_out/prof -name "*.csv" | head -20

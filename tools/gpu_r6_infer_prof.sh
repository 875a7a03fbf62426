# the headline's kernel stats on the current tree: rocprofv3 --kernel-trace --stats of bench.py's
# inference legs (fp16 headline + bf16), no training legs; + the forward_pair test
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/infer
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_disc.py > gpurun_out/infer/t.log 2>&1 || { tail -30 gpurun_out/infer/t.log; exit 1; }
tail -1 gpurun_out/infer/t.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/infer/kt -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-train --no-stress --no-cpu-baseline > gpurun_out/infer/bench.json 2> gpurun_out/infer/bench.err
tail -1 gpurun_out/infer/bench.json | cut -c1-400

# round-end sequence: full -m gpu suite, smoke, bench line, then the configs[2] / configs[3] kernel
# breakdowns (tools/gpu_r6_legprof.sh)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh
bash tools/gpu_r6_legprof.sh > gpurun_out/legprof.txt 2>&1
echo LEGPROF_OK

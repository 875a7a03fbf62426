# Product library vs csrc/build_var variants: the chain / strip tests on the product, then the
# inference bench leg per library, interleaved x2 (and TRAIN=1: the stage-1 step)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/libab
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_group_chain.py tests/test_gpu_northstar.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/libab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/libab/tests.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for l in face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null); do
  FEN_HIP_LIB=$l timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 40 --warmup 5 > gpurun_out/libab/b.json 2> gpurun_out/libab/b.log || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/libab/b.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['bf16']['value'])" $(basename $l)
  if [ "${TRAIN:-0}" = "1" ]; then
    FEN_HIP_LIB=$l STEPS=30 timeout -k 10 200 python tools/train_step.py > gpurun_out/libab/ts.log 2>&1 || exit 1
    echo "   $(tail -1 gpurun_out/libab/ts.log)"
  fi
done
done

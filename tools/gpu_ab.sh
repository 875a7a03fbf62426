# Same-box A/B of library variants (one parameterised script; replaces round 5's single-use
# gpu_batch_r5*.sh).  Run from the repo root through gpurun, e.g.
#   VARIANTS="prod vgg2" TESTS="tests/test_gpu_vgg.py" CMD="python tools/train_step.py" \
#     CMD_ENV="PERCEPTUAL=1 STEPS=20" REPS=3 bash tools/gpu_ab.sh
# VARIANTS  names: "prod" = the product library, anything else = build_var/libfen_hip_<name>.so
#           (make -C face-super-resolution_amd/csrc variant V=<name> DEFS=...)
# TESTS     pytest files run once per variant first (a variant that breaks parity stops the run)
# CMD       the timing command (its last stdout line is reported), CMD_ENV extra env for it,
#           REPS repetitions interleaved over the variants (same box, alternating order)
# CONFIGS   alternatively ';'-separated environment settings A/B'd on the product library
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
V=face-super-resolution_amd/csrc/build_var
lib_of() { if [ "$1" = prod ]; then echo face-super-resolution_amd/src/hip/libfen_hip.so; else echo $V/libfen_hip_$1.so; fi; }
REPS=${REPS:-3}
if [ -n "$CONFIGS" ]; then IFS=';' read -ra ITEMS <<< "$CONFIGS"; else read -ra ITEMS <<< "${VARIANTS:-prod}"; fi
envfor() { if [ -n "$CONFIGS" ]; then echo "$1"; else echo "FEN_HIP_LIB=$(lib_of $1)"; fi; }
if [ -n "$TESTS" ]; then
  for it in "${ITEMS[@]}"; do
    tag=$(echo "$it" | tr -c 'A-Za-z0-9_\n' '_')
    env $(envfor "$it") timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/ab/t_$tag.log 2>&1
    rc=$?; echo "[$it] tests rc=$rc: $(tail -1 gpurun_out/ab/t_$tag.log)"
    [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/ab/t_$tag.log | head -8; exit $rc; }
  done
fi
[ -n "$CMD" ] || exit 0
for rep in $(seq 1 $REPS); do
  for it in "${ITEMS[@]}"; do
    env $(envfor "$it") $CMD_ENV timeout -k 10 ${CMD_TIMEOUT:-300} $CMD > gpurun_out/ab/cmd.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "[$it] cmd rc=$rc"; tail -8 gpurun_out/ab/cmd.log; exit $rc; }
    echo "rep $rep [$it] $(tail -1 gpurun_out/ab/cmd.log)"
  done
done

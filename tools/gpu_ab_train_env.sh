# Same-box A/B of environment switches on the stage-1 training step (tools/train_step.py,
# graph-replayed, B=32): every configuration of $AB_CONFIGS (';'-separated, each a list of
# VAR=value) in turn, $REPS rounds.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra CFGS <<< "${AB_CONFIGS:-FEN_WGRAD_SIDE=0;FEN_WGRAD_SIDE=1}"
for r in $(seq 1 ${REPS:-2}); do
  for v in "${CFGS[@]}"; do
    echo "$v | $(env $v STEPS=${STEPS:-30} timeout -k 10 300 python tools/train_step.py 2>/dev/null | tail -1)"
  done
done

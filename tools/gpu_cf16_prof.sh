# per-kernel durations of the conv_first forward forms on the perceptual step (FEN_CF_M16=0/1)
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 1; do
  FEN_CF_M16=$v PERCEPTUAL=1 STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cf16_$v -o run --output-format csv -- python tools/train_step.py > gpurun_out/cf16_$v.log 2>&1
  f=$(find gpurun_out/cf16_$v -name '*kernel_stats.csv' | head -1)
  grep -i "conv_first" "$f" | cut -c1-160
done

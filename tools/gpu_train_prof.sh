# Per-kernel breakdown of the stage-1 training step (tools/train_step.py under rocprofv3).
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tp
timeout -k 10 200 python tools/train_step.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp/prof -o run --output-format csv -- python tools/train_step.py > gpurun_out/tp/prof.log 2>&1
python tools/prof_summary.py stats "$(find gpurun_out/tp/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/tp/train_kernel_stats.csv > /dev/null
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/tp/train_kernel_stats.csv")))
n = 24  # replays: 20 timed + 3 warm-up + 1 capture warm-up
tot = sum(float(r["TotalDurationNs"]) for r in rows) / n / 1e3
print(f"per step (kernel time): {tot:.1f} us")
for r in rows[:28]:
    print(f'{float(r["TotalDurationNs"]) / n / 1e3:8.1f} us/step {int(r["Calls"]) / n:6.1f} x {float(r["AverageNs"]) / 1e3:8.2f} us  {r["Name"][:90]}')
PY

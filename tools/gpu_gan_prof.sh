set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gan
timeout -k 10 300 python tools/gan_step.py
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gan/prof -o run --output-format csv -- python tools/gan_step.py > gpurun_out/gan/prof.log 2>&1
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/gan/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
NIT = 15   # gan_step.py with STEPS=5: 3 + 5 eager, then 2 eager + 5 replays (the capture runs nothing)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"all kernels: {tot / NIT / 1e6:.2f} ms per iteration ({NIT} iterations), {calls / NIT:.0f} launches per iteration")
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:15]:
    print(f'{float(r["TotalDurationNs"]) / NIT / 1e3:9.1f} us/it {int(r["Calls"]) / NIT:7.1f} x {float(r["AverageNs"]) / 1e3:8.2f} us  {r["Name"][:80]}')
PY

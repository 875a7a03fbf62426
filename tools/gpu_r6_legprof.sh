# Round 6: kernel breakdown of BASELINE configs[2] (stage-1 L1 + perceptual, B=32) and configs[3]
# (stage-3 GAN iteration, B=16): rocprofv3 --kernel-trace --stats of the replayed step alone.
# Outputs gpurun_out/r6prof/{perc,gan}/..., summarised to gpurun_out/r6prof/*.txt
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6prof
PERCEPTUAL=1 STEPS=10 timeout -k 10 300 python tools/train_step.py
PERCEPTUAL=1 STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6prof/perc -o run --output-format csv -- python tools/train_step.py > gpurun_out/r6prof/perc.log 2>&1
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6prof/gan -o run --output-format csv -- python tools/gan_step.py > gpurun_out/r6prof/gan.log 2>&1
python - <<'PY'
import csv, glob
for leg, nit in (("perc", 14), ("gan", 15)):
    f = glob.glob(f"gpurun_out/r6prof/{leg}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    calls = sum(int(r["Calls"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    with open(f"gpurun_out/r6prof/{leg}.txt", "w") as o:
        print(f"{leg}: all kernels {tot / nit / 1e6:.3f} ms per step ({nit} steps), {calls / nit:.1f} launches per step", file=o)
        for r in rows[:40]:
            print(f'{float(r["TotalDurationNs"]) / nit / 1e3:9.1f} us/step {int(r["Calls"]) / nit:7.2f} x {float(r["AverageNs"]) / 1e3:8.2f} us  {r["Name"][:110]}', file=o)
    print(open(f"gpurun_out/r6prof/{leg}.txt").read())
PY

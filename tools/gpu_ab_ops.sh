# Per-launch A/B: parity tests on the product library, then tools/op_times.py (inference and
# TRAIN=1) for the product library and every csrc/build_var variant, interleaved x2, then the
# inference bench leg per library and (STAMPS=1) the strip stamps of the product build.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abops
if [ "${TESTS:-}" != "none" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_group_strip.py tests/test_gpu_group_strip_bwd.py tests/test_gpu_kernels.py tests/test_gpu_northstar.py} \
    -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abops/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/abops/tests.log
[ $rc -eq 0 ] || exit 1
fi
libs="face-super-resolution_amd/src/hip/libfen_hip.so $(ls face-super-resolution_amd/csrc/build_var/libfen_hip_*.so 2>/dev/null)"
IFS=';' read -ra ENVS <<< "${AB_ENVS:-X=0}"
for rep in 1 2; do
  for l in $libs; do
   for e in "${ENVS[@]}"; do
    n=$(basename $l .so)_$(echo $e | tr '=' '-')
    FEN_HIP_LIB=$l timeout -k 10 200 env $e python tools/op_times.py > gpurun_out/abops/inf_${n}_$rep.txt 2>&1 || { echo "op_times $n failed"; exit 1; }
    FEN_HIP_LIB=$l TRAIN=1 timeout -k 10 300 env $e python tools/op_times.py > gpurun_out/abops/trn_${n}_$rep.txt 2>&1 || { echo "op_times train $n failed"; exit 1; }
    python - gpurun_out/abops/inf_${n}_$rep.txt gpurun_out/abops/trn_${n}_$rep.txt "$n r$rep" <<'PY'
import sys, re
def rows(f):
    out = {}
    for l in open(f):
        m = re.match(r"\s*\d+ (\S+)\s+(.*?)\s+([\d.]+) us", l)
        if m:
            k = (m.group(1) + " " + m.group(2)).strip()
            out.setdefault(k, []).append(float(m.group(3)))
        if l.startswith("sum of launches"):
            out["SUM"] = [float(l.split()[3])]
    return out
i, t = rows(sys.argv[1]), rows(sys.argv[2])
gi = [v for k, v in i.items() if k.startswith("group_strip ")][0][0]
up = [v for k, v in i.items() if "128x128 epi=7" in k][0][0]
gf = [v for k, v in t.items() if k.startswith("group_strip ")]
gb = [v for k, v in t.items() if k.startswith("group_strip_bwd")]
wg = [x for k, v in t.items() if k.startswith("wgrad3x3_multi") for x in v]
cl = [v for k, v in t.items() if k.startswith("conv_last_dgrad")]
print(f"{sys.argv[3]:24s} inf: strip {gi:7.1f} up1 {up:6.1f} sum {i['SUM'][0]:7.1f} | train: strip fwd {gf[0][0] if gf else 0:7.1f} "
      f"bwd {gb[0][0] if gb else 0:7.1f} wg {sum(wg) / max(len(wg), 1):6.1f} cld {cl[0][0] if cl else 0:6.1f} sum {t['SUM'][0]:7.1f}")
PY
    FEN_HIP_LIB=$l STEPS=20 timeout -k 10 200 env $e python tools/train_step.py > gpurun_out/abops/ts.log 2>&1 || { echo "train_step $n failed"; tail -5 gpurun_out/abops/ts.log; exit 1; }
    echo "   $(tail -1 gpurun_out/abops/ts.log)"
   done
  done
done
for l in $libs; do
  FEN_HIP_LIB=$l timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 30 --warmup 5 > gpurun_out/abops/b.json 2> gpurun_out/abops/b.log || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/abops/b.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $(basename $l)
done
if [ "${STAMPS:-0}" = "1" ]; then
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so timeout -k 10 200 python tools/stamp_strip.py 2>&1 | grep -v amdgpu.ids
fi

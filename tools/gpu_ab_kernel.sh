# Same-box A/B of the dominant kernel: the library at HEAD (build_var/libfen_hip_base.so with
# the HEAD descriptor, tools/pmc_rcab_base.py) against the working tree, per-launch time of
# one deferred RCAB under rocprofv3 --stats (fp16 / bf16), then the inference bench of each.
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
BASE=face-super-resolution_amd/csrc/build_var/libfen_hip_base.so
kt() {  # name script env...
  local n=$1 sc=$2; shift 2
  for p in fp16 bf16; do
    env "$@" PREC=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$n-$p -o run --output-format csv -- python $sc > gpurun_out/ab/$n-$p.log 2>&1
    f=$(find gpurun_out/ab/$n-$p -name '*kernel_stats.csv' | head -1)
    python -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'k_rcab' in x['Name']]; print('$n $p', [(x['Calls'], round(float(x['AverageNs'])/1e3,2), round(float(x['MinNs'])/1e3,2)) for x in r])"
  done
}
kt base tools/pmc_rcab_base.py FEN_HIP_LIB=$BASE
kt new tools/pmc_rcab.py
kt base2 tools/pmc_rcab_base.py FEN_HIP_LIB=$BASE
kt new2 tools/pmc_rcab.py

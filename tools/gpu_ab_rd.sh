# A/B of rcab_deferred variants (build_var/libfen_hip_<V>.so): phase stamps and live per-launch time
# VARIANTS: stamp builds (st_*), TVARIANTS: timing builds ('base' = the product library)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for V in ${VARIANTS:-st}; do
  echo "== stamps $V"
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_var/libfen_hip_$V.so timeout -k 10 100 python tools/stamp_rcab_d.py 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-2000 || exit 1
done
for V in ${TVARIANTS:-base}; do
  L=face-super-resolution_amd/csrc/build_var/libfen_hip_$V.so
  [ "$V" = base ] && L=face-super-resolution_amd/src/hip/libfen_hip.so
  echo "== timing $V"
  FEN_HIP_LIB=$L MODES=deferred timeout -k 10 100 python tools/bench_rcab_modes.py 2>&1 | grep -v amdgpu.ids || exit 1
done

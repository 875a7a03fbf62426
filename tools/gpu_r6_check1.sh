# round 6: ADVICE / D256 / SSIM fallback parity on the GPU, the streamed conv's counters on a VGG shape, bench
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_vgg
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_ssim.py tests/test_gpu_rccl.py tests/test_gpu_gan_capture.py tests/test_gpu_dp_engine.py "tests/test_gpu_bench_legs.py::test_gan_leg_d256_matches_cpu_replay" -s > gpurun_out/g1_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/g1_tests.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/g1_tests.log | head; exit $rc; }
timeout -k 10 120 python tools/bench_vgg_conv.py > gpurun_out/g1_vggconv.txt 2>&1 || exit 1
cat gpurun_out/g1_vggconv.txt
for set in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc_vgg/p$i -o run --output-format csv -- python tools/pmc_vggconv.py > gpurun_out/pmc_vgg/log$i.txt 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/pmc_vgg/log$i.txt; exit 1; }
done
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_vgg/kt -o run --output-format csv -- python tools/pmc_vggconv.py > gpurun_out/pmc_vgg/logkt.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-stress --no-cpu-baseline > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/g1_bench.err; exit $rc

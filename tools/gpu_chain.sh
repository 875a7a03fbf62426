export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chain
timeout -k 10 300 python -u -m pytest tests/test_gpu_group_chain.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/chain/t1.log 2>&1
rc=$?; echo "chain tests rc=$rc"; tail -25 gpurun_out/chain/t1.log | grep -E "PASS|FAIL|Error|error|passed|failed" | head -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_northstar.py tests/test_gpu_group_strip.py tests/test_gpu_train64.py tests/test_gpu_net.py tests/test_gpu_module.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/chain/t2.log 2>&1
rc=$?; echo "northstar rc=$rc"; tail -3 gpurun_out/chain/t2.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for v in ${AB_ENVS:-FEN_CHAIN_AFTER_BODY=1 FEN_CHAIN_AFTER_BODY=0}; do
env $v timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --no-stress --steps 40 --warmup 5 > gpurun_out/chain/b.json 2> gpurun_out/chain/b.log || exit 1
python -c "import json,sys; d=json.loads(open('gpurun_out/chain/b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['bf16']['value'])"
done
done

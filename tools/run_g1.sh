cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/${TAG:-g1}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG:-g1}/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG:-g1}/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG:-g1}/bench.log 2>&1 || exit $?
cat gpurun_out/${TAG:-g1}/bench.log | tail -1

#!/bin/bash
# GPU test run of round 3: the -m gpu suite (stops after 10 failures), then a
# short bench line.  TAG names the gpurun_out/ subdirectory.
cd ${GRAFT_REPO_ROOT:-/root/repo}
D=gpurun_out/${TAG:-r3}
mkdir -p $D
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v --maxfail=10 --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > $D/pytest.log 2>&1; rc=$?
tail -15 $D/pytest.log
[ $rc -le 1 ] || exit $rc
if [ -n "${BENCH:-}" ]; then
    timeout -k 10 400 python -u bench.py $BENCH > $D/bench.log 2>&1 || exit $?
    tail -c 3000 $D/bench.log
fi
exit $rc

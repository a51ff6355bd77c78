#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that crashes / times out (exit code not 0 or 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "=== $name" ; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc"; tail -n 25 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
    return 0
}
run pytest_gpu 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py ${BENCH_ARGS}
if [ -n "$PROFILE" ]; then
    export TMPDIR=/tmp
    ROOTDIR=$(pwd)
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/$OUT/prof" -o run \
        --output-format csv -- python3 "$ROOTDIR/bench.py" --steps 5 --warmup 2 --no-cpu-baseline \
        > "$ROOTDIR/$OUT/rocprof.log" 2>&1); rc=$?
    echo "rocprof rc=$rc"; tail -n 5 "$OUT/rocprof.log"
fi

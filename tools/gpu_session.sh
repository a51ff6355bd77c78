#!/bin/bash
# One GPU session on the gpurun box, steps chosen by name, each under its own
# time limit, stopping at the first failure:
#   TAG=name bash tools/gpu_session.sh tests[=<-k expr>] smoke bench[=<args>] py=<script args> prof=<script args>
#   tests      pytest -m gpu (optionally -k <expr>)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py [args]
#   py         python -u tools/<script> [args]
#   sh         bash tools/<script> [args]
#   prof       rocprofv3 --kernel-trace --stats over python3 tools/<script> [args]
# Output under gpurun_out/$TAG/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); T=${TAG:-s}; OUT=$R/gpurun_out/$T; mkdir -p "$OUT"; export TMPDIR=/tmp
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
n=0
for step in "$@"; do
  n=$((n+1)); name=${step%%=*}; arg=""; [[ "$step" == *=* ]] && arg=${step#*=}
  case "$name" in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread "${K[@]}" \
          > "$OUT/pytest_gpu_$n.log" 2>&1 \
          || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/pytest_gpu_$n.log" | tail -20; exit 1; }
      tail -1 "$OUT/pytest_gpu_$n.log";;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
          || { echo "smoke rc=$?"; tail -5 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log";;
    bench)
      timeout -k 10 600 python bench.py $arg > "$OUT/bench_$n.log" 2>&1 \
          || { echo "bench rc=$?"; tail -5 "$OUT/bench_$n.log"; exit 1; }
      tail -1 "$OUT/bench_$n.log" | cut -c1-400;;
    py)
      timeout -k 10 600 python -u tools/$arg > "$OUT/py_$n.log" 2>&1 \
          || { echo "py rc=$?"; tail -15 "$OUT/py_$n.log"; exit 1; }
      tail -40 "$OUT/py_$n.log";;
    sh)
      timeout -k 10 900 bash tools/$arg > "$OUT/sh_$n.log" 2>&1 \
          || { echo "sh rc=$?"; tail -15 "$OUT/sh_$n.log"; exit 1; }
      tail -40 "$OUT/sh_$n.log";;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o run --output-format csv \
          -- python3 "$R/tools/"$arg > "$OUT/prof_$n.log" 2>&1) \
          || { echo "prof rc=$?"; tail -15 "$OUT/prof_$n.log"; exit 1; }
      tail -5 "$OUT/prof_$n.log";;
    *) echo "unknown step $name"; exit 2;;
  esac
done
echo "session done"

#!/bin/bash
# Same-box A/B over environment settings (a library is one too:
# O3DML_AMD_LIB=<path>), every configuration run twice, interleaved:
#   bash tools/ab.sh KIND ENV1=a,ENV2=b ENV1=c ...   (a comma joins the settings of one configuration)
# KIND:
#   frs     C1 FRS bench line (bench.py, FRS only): Mpts/s, ms/step, search / row-copy kernel ms
#   bench   whole bench.py (no CPU legs, no sweep; BENCH_ARGS appended): C1, RandLA, SCN, C3, C5
#   randla  RandLA-Net section (FRAMES scans, default 4): frames/s warm and cold
#   scn     SparseConvUnet eval frames (tools/scn_frames.py 20)
#   gemm    sparse-conv GEMM probe (tools/gemm_probe.py; SHAPES / REPS from the caller)
#   knn     batched k = 16 kNN at RandLA-Net's shapes (tools/knn_probe.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
KIND=$1; shift
NOSEC="--no-cpu-baseline --sweep-reps 0 --op-reps 0"
run() {
  case "$KIND" in
    frs)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 $NOSEC --randla-frames 0 --sparse-conv-reps 0 \
          --kpconv-steps 0 --pointpillars-steps 0 2>/dev/null | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('Mpts/s', d['value'], 'ms/step', d['ms_per_step'], 'kernels', d['roofline'].get('kernel_ms_all'))";;
    bench)
      timeout -k 10 400 python bench.py $NOSEC ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
def g(*k):
    v = d
    for x in k:
        v = v.get(x, {}) if isinstance(v, dict) else None
    return v
print('C1', d['value'], 'RandLA fps', g('randlanet', 'frames_per_s'), 'SCN ms', g('sparse_conv', 'unet', 'ms_per_frame'),
      'C3 ms', g('kpconv', 'ms_per_step'), 'C5 ms', g('pointpillars', 'ms_per_step'))";;
    randla)
      timeout -k 10 300 python bench.py --steps 1 --warmup 1 $NOSEC --randla-frames "${FRAMES:-4}" \
          --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 2>/dev/null | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())['randlanet']
print('frames/s', d['frames_per_s'], 'ms/frame', d['ms_per_frame'], 'cold', d['cold_frames_per_s'])";;
    scn) timeout -k 10 120 python tools/scn_frames.py 20 2>/dev/null | grep "SCN frame";;
    gemm) timeout -k 10 120 python tools/gemm_probe.py 2>/dev/null | grep -v "^$";;
    knn) timeout -k 10 120 python tools/knn_probe.py 2>/dev/null | grep -v "^$" | tail -3;;
    *) echo "unknown kind $KIND"; return 2;;
  esac
}
for rep in 1 2; do
  for cfg in "$@"; do
    echo "== $cfg (rep $rep)"
    export_env=${cfg//,/ }
    (export $export_env; run) || exit 1
  done
done

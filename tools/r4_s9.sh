#!/bin/bash
# Round-4 session 9: A/B of the radix tile size (lib_rs16 / lib_rs32 full
# rebuilds) on the 2^24 single scene, the FRS bench line and SCN frames; SCN
# frames with the split-K reduce folded into the GEMM (host-bound eval); the
# BN finalize modes on the C3 step; RandLA frames/s.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s9
for m in 1 2; do
  O3DML_BN_FINALIZE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_batchnorm.py -q --timeout 120 --timeout-method thread > gpurun_out/r4s9/bn$m.log 2>&1 \
      || { grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r4s9/bn$m.log | head; exit 1; }
  echo "BN_FINALIZE=$m tests: $(tail -1 gpurun_out/r4s9/bn$m.log)"
done
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0 --kpconv-steps 10"
for e in 0 1 2 0 1 2; do
  O3DML_BN_FINALIZE=$e timeout -k 10 200 python bench.py $A > gpurun_out/r4s9/kp.log 2>&1 || { tail -5 gpurun_out/r4s9/kp.log; exit 1; }
  echo "BN_FINALIZE=$e $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s9/kp.log').read().strip().splitlines()[-1]);k=d['kpconv'];print(k['ms_per_step'], k['ms_collate'])")"
done
for lib in lib lib_rs16 lib_rs32; do
  L=$PWD/open3d-ml_amd/$lib/libo3dml_amd.so
  a=$(O3DML_AMD_LIB=$L timeout -k 10 120 python tools/frs_big_time.py 24 5) || { echo "$lib big rc=$?"; exit 1; }
  b=$(O3DML_AMD_LIB=$L timeout -k 10 120 python tools/scn_frames.py 20) || { echo "$lib scn rc=$?"; exit 1; }
  echo "$lib | $a | $b"
done
for e in 0 1 0 1; do
  echo "GEMM_FUSED_REDUCE=$e $(O3DML_GEMM_FUSED_REDUCE=$e timeout -k 10 120 python tools/scn_frames.py 20)" || exit 1
done
timeout -k 10 200 python bench.py --steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 --randla-frames 6 > gpurun_out/r4s9/rl.log 2>&1 || exit 1
echo "randla fps $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s9/rl.log').read().strip().splitlines()[-1]);print(d['randlanet']['frames_per_s'])")"

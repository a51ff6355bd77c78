#!/bin/bash
# Round-4 session 9: A/B of the radix tile size (lib_rs16 / lib_rs32 full
# rebuilds) on the 2^24 single scene, the FRS bench line and SCN frames; and
# SCN frames with the split-K reduce folded into the GEMM (host-bound eval).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s9
for rep in 1 2; do
  for lib in lib lib_rs16 lib_rs32; do
    L=$PWD/open3d-ml_amd/$lib/libo3dml_amd.so
    a=$(O3DML_AMD_LIB=$L timeout -k 10 120 python tools/frs_big_time.py 24 5) || { echo "$lib big rc=$?"; exit 1; }
    b=$(O3DML_AMD_LIB=$L timeout -k 10 120 python tools/scn_frames.py 20) || { echo "$lib scn rc=$?"; exit 1; }
    echo "$lib | $a | $b"
  done
done
bash tools/ab_libs_frs.sh lib lib_rs16 lib_rs32 || exit 1
for e in 0 1 0 1; do
  echo "FUSED_REDUCE=$e $(O3DML_GEMM_FUSED_REDUCE=$e timeout -k 10 120 python tools/scn_frames.py 20)" || exit 1
done
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0 --kpconv-steps 10"
for e in 1 0 1 0; do
  O3DML_BN_LAST_BLOCK=$e timeout -k 10 200 python bench.py $A > gpurun_out/r4s9/kp.log 2>&1 || { tail -5 gpurun_out/r4s9/kp.log; exit 1; }
  echo "BN_LAST_BLOCK=$e $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s9/kp.log').read().strip().splitlines()[-1]);k=d['kpconv'];print(k['ms_per_step'], k['ms_collate'])")"
done
timeout -k 10 200 python bench.py --steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 --randla-frames 6 > gpurun_out/r4s9/rl.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r4s9/rl.log').read().strip().splitlines()[-1]);print(d['randlanet']['frames_per_s'])"

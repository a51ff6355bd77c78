cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s5
for e in "O3DML_KPCONV_MFMA=1 O3DML_FUSED_BN=1" "O3DML_KPCONV_MFMA=0 O3DML_FUSED_BN=1" "O3DML_KPCONV_MFMA=1 O3DML_FUSED_BN=0" "O3DML_KPCONV_MFMA=0 O3DML_FUSED_BN=0"; do
  env $e timeout -k 10 200 python -u -m pytest tests/test_gpu_kpfcnn.py -q --timeout 120 --timeout-method thread -k "step_matches" > gpurun_out/r4s5/ab.log 2>&1
  echo "$e: $(grep -E 'AssertionError: \(|passed|failed' gpurun_out/r4s5/ab.log | tr '\n' ' ')"
done
exit 0

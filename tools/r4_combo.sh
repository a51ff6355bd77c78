bash tools/r4_s9.sh > gpurun_out/r4s9.log 2>&1; echo "s9 rc=$?"; tail -30 gpurun_out/r4s9.log
TAG=r4fin1 bash tools/r4_final.sh

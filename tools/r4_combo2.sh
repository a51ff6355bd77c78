#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/r4_s11.sh || exit 1
bash tools/r4_s10.sh

#!/bin/bash
# Round-4 FRS cost split: per library build (main + O3DML_DIAG variants) one
# SQ instruction-count PMC pass of the FRS-only bench, then interleaved
# FRS-only bench lines (kernel times).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc_variants.sh "$@" || exit 1
libs=""
for v in "$@"; do if [ "$v" = main ]; then libs="$libs lib"; else libs="$libs lib_$v"; fi; done
bash tools/ab_libs_frs.sh $libs

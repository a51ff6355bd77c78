#!/bin/bash
# PMC passes (one counter group per process, kernel-trace only) over ${PROBE:-tools/frs_probe.py}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$ROOTDIR/${PROBE:-tools/frs_probe.py}" > "$OUT/p$i.log" 2>&1)
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<< "${GROUPS_LIST}"

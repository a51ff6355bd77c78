"""Summarise a tools/round_profile.sh run into profiles/<round>/:
kernel stats CSV copy + pmc_<kernel>.json with HBM bytes per launch
(2 x FETCH_SIZE per the gfx950 calibration in MI355X_MICROARCH.md §HBM, plus
WRITE_SIZE; both reported by rocprofv3 in KiB) and the SQ counters.
usage: python tools/pmc_traffic.py gpurun_out/<tag> profiles/r01 frs_group_kernel<1, false, false, 0"""
import glob
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main(src, dst, match, name):
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "stats", "**", "run_kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{name}_kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "bench.log")):  # (PMC passes over a probe have none)
        shutil.copy(os.path.join(src, "bench.log"), os.path.join(dst, f"{name}_bench.log"))
    res = load(src, match)
    assert len(res) == 1, list(res)
    (kname, c), = res.items()
    fetch = 2 * c["FETCH_SIZE"] * 1024
    write = c["WRITE_SIZE"] * 1024
    out = {"kernel": kname, "hbm_bytes_per_launch": int(fetch + write), "read_bytes_2x_fetch_size": int(fetch),
           "write_bytes": int(write), "counters_per_launch": c,
           "note": "FETCH_SIZE doubled (gfx950 reports half of wide streaming reads); access widths other than "
                   "16 B/lane are uncalibrated per the guide, so treat as an estimate"}
    with open(os.path.join(dst, f"pmc_{name}.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: out[k] for k in ("kernel", "hbm_bytes_per_launch", "read_bytes_2x_fetch_size",
                                          "write_bytes")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else "frs")

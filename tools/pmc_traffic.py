"""Summarise rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of one bench frame into the traffic record
bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py gpurun_out/TAG_pmc_fetch gpurun_out/TAG_pmc_write OUT.json [--config C3]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch, from the L2's memory-side request counters (Infinity Cache
hits included).  /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports half the
bytes of 16 B/lane reads, so the fetch figure is doubled; WRITE_SIZE is taken as is.  Other access widths
are uncalibrated, so the record keeps the raw counters beside the corrected bytes.
"""
import csv
import glob
import json
import os
import subprocess
import sys

KERNEL = "rpk::render_kernel<false, "  # the frame kernel (either stack variant), not the probe


def counter(dirname, name):
    vals = []
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == name and KERNEL in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for {KERNEL} under {dirname}")
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "C3"
    fetch_kib, nf = counter(fetch_dir, "FETCH_SIZE")
    write_kib, nw = counter(write_dir, "WRITE_SIZE")
    rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    rec = {
        "kernel": KERNEL, "config": config, "git": rev, "dispatches": [nf, nw],
        "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
        "fetch_bytes": 2.0 * fetch_kib * 1024.0, "write_bytes": write_kib * 1024.0,
        "traffic_bytes": 2.0 * fetch_kib * 1024.0 + write_kib * 1024.0,
        "note": "per dispatch of the frame kernel; FETCH_SIZE doubled per the gfx950 correction",
    }
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()

"""Summarise an interleaved A/B session of tools/gpu_session.sh (steps ab_<CFG>): per config and run the ms/frame
of each rep, the median and the change against the base run; with --out, also a record for profiles/ that carries
the session's commands (gpurun_out/<tag>_manifest.txt) next to the numbers.

    python tools/ab_summary.py r4n [--base main] [--out profiles/r4/x_ab.json --what "..." --session "..."]
"""
import argparse
import glob
import json
import os
import re
import statistics
from collections import defaultdict


def collect(tag):
    runs = defaultdict(lambda: defaultdict(list))  # cfg -> run -> [ms]
    for f in sorted(glob.glob(f"gpurun_out/{tag}_*_*.json")):
        m = re.match(rf"gpurun_out/{re.escape(tag)}_(C\d)_(.+)_(\d+)\.json$", f)
        if not m:
            continue
        try:
            line = open(f).read().strip().splitlines()[-1]
            runs[m.group(1)][m.group(2)].append(json.loads(line)["ms_per_step"])
        except Exception:
            pass
    return runs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--base", default="main")
    ap.add_argument("--out")
    ap.add_argument("--what", default="")
    ap.add_argument("--session", default="")
    a = ap.parse_args()
    runs = collect(a.tag)
    rec = {"what": a.what, "session": a.session, "ms_per_frame": {}, "delta_pct_vs_" + a.base: {}, "commands": {}}
    for cfg, by in runs.items():
        base = statistics.median(by[a.base]) if a.base in by else None
        for name, v in by.items():
            med = statistics.median(v)
            d = None if base is None else round(100 * (med / base - 1), 2)
            rec["ms_per_frame"][f"{cfg}_{name}"] = {"reps": v, "median": med}
            rec["delta_pct_vs_" + a.base][f"{cfg}_{name}"] = d
            print(f"{a.tag:6s} {cfg} {name:10s} median {med:9.2f} ms  ({'' if d is None else f'{d:+.2f} %'})  reps {v}")
    man = f"gpurun_out/{a.tag}_manifest.txt"
    if os.path.exists(man):
        for line in open(man):
            k, _, v = line.partition(": ")
            if re.search(r"_1\.json$", k) or "pmc" in k:
                rec["commands"][k.split("/")[-1]] = v.strip()
    if a.out:
        json.dump(rec, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

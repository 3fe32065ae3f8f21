"""Summarise A/B runs (tools/gpu_ab_r3.sh outputs): per variant the ms/frame of each rep, the median, and the
change against the first variant."""
import glob, json, re, statistics, sys
from collections import defaultdict

for tag in sys.argv[1:]:
    runs = defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/{tag}_*.json")):
        m = re.match(rf"gpurun_out/{re.escape(tag)}_(.+)_(\d+)\.json$", f)
        if not m:
            continue
        try:
            runs[m.group(1)].append(json.load(open(f))["ms_per_step"])
        except Exception:
            pass
    base = None
    for name, v in runs.items():
        med = statistics.median(v)
        base = base or med
        print(f"{tag:12s} {name:14s} median {med:9.2f} ms  ({100 * (med / base - 1):+.2f} %)  reps {v}")

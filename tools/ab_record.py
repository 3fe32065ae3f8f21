"""Append one interleaved A/B session (tools/gpu_abrun.sh output) to profiles/r2/ab_sweeps.json.

    python tools/ab_record.py ab29 "what was compared" gpurun_out/q1_*.json
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    key, what, files = sys.argv[1], sys.argv[2], sys.argv[3:]
    path = os.path.join(REPO, "profiles", "r2", "ab_sweeps.json")
    rec = json.load(open(path))
    results = {}
    for f in sorted(files):
        label = os.path.basename(f)[:-5].split("_", 1)[1]
        d = json.load(open(f))
        results[label] = {"config": d["config"]["workload"].split(":")[0], "ms_per_frame": d["ms_per_step"],
                          "rays_per_frame": d["config"]["rays_per_frame"],
                          "scene_options": d["config"]["scene_options"]}
    rec["runs"][key] = {"what": what, "results": results}
    json.dump(rec, open(path, "w"), indent=1)
    for k, v in results.items():
        print(f"{k:12s} {v['config']} {v['ms_per_frame']:9.2f} ms  {v['scene_options']}")


if __name__ == "__main__":
    main()

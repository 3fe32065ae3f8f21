"""Distribution of the longest measured unit per tile (product build, not the diagnostic one): a whole frame renders,
then the workspace's measured tile costs (rp_workspace_tile_costs: per tile the summed and the longest duration of the
one unit in eight the render times, 100 MHz ticks >> MEAS_SHIFT) give how long the slowest (pixel, sample batch) units
run against the frame and against an N-way shard's frame -- the latency a frame's tail, and a frame in flight, waits on.

    python tools/unit_times.py [--config C3] [--frames 2]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]
MEAS_SHIFT = 6  # rp_kernel.h
TICK_MS = (1 << MEAS_SHIFT) / 1e5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    options = {}
    for kv in a.opt:
        k, v = kv.split("=", 1)
        options[k] = v if not v.lstrip("-").isdigit() else int(v)
    scene, params = scenes.config_scene(a.config)
    ds = DeviceScene(scene, options=options)
    out = {"config": a.config, "scene_options": options or "defaults", "frames": []}
    for _ in range(a.frames):
        _, _, st = ds.render(params)
        c = ds.tile_costs(params)  # (2, tiles): summed, longest (of the measured 1-in-8 units)
        mx = c[1].astype(np.float64) * TICK_MS
        units_per_tile = params.tile_w * params.tile_h * max(1, -(-params.spp // 32)) / 8.0
        mean_unit = c[0].astype(np.float64) * TICK_MS / units_per_tile
        q = np.percentile(mx, [50, 90, 99, 99.9, 100])
        out["frames"].append({
            "frame_ms": round(st["seconds"] * 1e3, 2),
            "mean_unit_ms": round(float(mean_unit.mean()), 3),
            "tile_longest_unit_ms_p50_p90_p99_p999_max": [round(float(x), 2) for x in q],
            "tiles_with_a_unit_over_10ms": int((mx > 10).sum()), "tiles": int(len(mx)),
            "longest_tile": int(np.argmax(mx))})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

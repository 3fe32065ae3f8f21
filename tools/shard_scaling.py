"""Strong-scaling projection on ONE GPU: the per-rank work of an N-GPU run is one tile-interleaved shard
(tile t -> rank t % N), so rendering shard 0..N-1 of N one after another on one device measures every
rank's render time.  Projected N-GPU frame time = max over shards (+ the RCCL gather, not included);
efficiency = T(1) / (N * max_shard T(N)).  Diagnostic only; the driver's 8-GPU bench is the measurement.

    python tools/shard_scaling.py [--config C3] [--ns 1,2,4,8]
"""
import argparse
import json
import os
import sys
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--tile", type=int, default=0, help="square tile size (default: the config's)")
    a = ap.parse_args()
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    scene, params = scenes.config_scene(a.config)
    if a.tile:
        params = replace(params, tile_w=a.tile, tile_h=a.tile)
    ds = DeviceScene(scene)
    ds.render(replace(params, spp=4))  # warm
    out = {"config": a.config, "tile": [params.tile_w, params.tile_h], "per_n": {}}
    t1 = None
    for n in [int(x) for x in a.ns.split(",")]:
        times, rays = [], 0
        for s in range(n):
            _, _, st = ds.render(replace(params, shard=s, num_shards=n))
            times.append(st["seconds"])
            rays += st["rays"]
        tmax = max(times)
        if n == 1:
            t1 = tmax
        out["per_n"][n] = {"shard_seconds": [round(t, 4) for t in times], "max_s": round(tmax, 4),
                           "projected_mrays_s": round(rays / tmax / 1e6, 1),
                           "efficiency": round(t1 / (n * tmax), 3) if t1 else None}
        print(f"[shard_scaling] N={n} max {tmax:.4f}s", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

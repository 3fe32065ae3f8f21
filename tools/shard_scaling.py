"""Strong-scaling projection on ONE GPU: the per-rank work of an N-GPU run is one shard (tiles dealt by the
interleave t -> rank t % N, or by the balanced plan, RP_SHARD_BALANCED), so rendering shard 0..N-1 of N one after
another on one device measures every rank's render time (one frame in flight; the balanced plan's whole-frame
probe included).  Projected N-GPU frame time = max over shards (+ the RCCL gather, not included); balance =
max / mean shard time; efficiency = T(1) / (N * max_shard T(N)).  Diagnostic only; the driver's 8-GPU bench is
the measurement.

    python tools/shard_scaling.py [--config C3] [--ns 1,2,4,8] [--maps interleave,balanced] [--reps 3]
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
    ap.add_argument("--maps", default="interleave,balanced")
    ap.add_argument("--reps", type=int, default=3, help="renders per shard; the shard's time is their median")
    a = ap.parse_args()
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    scene, params = scenes.config_scene(a.config)
    if a.tile:
        params = replace(params, tile_w=a.tile, tile_h=a.tile)
    ds = DeviceScene(scene)
    ds.render(replace(params, spp=4))  # warm
    out = {"config": a.config, "tile": [params.tile_w, params.tile_h], "reps": a.reps, "per_map": {}}
    import statistics
    for mp in a.maps.split(","):
        smap = {"interleave": 0, "balanced": 1}[mp]
        per_n, t1 = {}, None
        for n in [int(x) for x in a.ns.split(",")]:
            times, rays = [], 0
            for s in range(n):
                reps = []
                for _ in range(a.reps):
                    _, _, st = ds.render(replace(params, shard=s, num_shards=n, shard_map=smap))
                    reps.append(st["seconds"])
                times.append(statistics.median(reps))
                rays += st["rays"]
            tmax = max(times)
            if n == 1:
                t1 = tmax
            per_n[n] = {"shard_seconds": [round(t, 4) for t in times], "max_s": round(tmax, 4),
                        "balance_max_over_mean": round(tmax / (sum(times) / n), 4),
                        "projected_mrays_s": round(rays / tmax / 1e6, 1),
                        "efficiency": round(t1 / (n * tmax), 3) if t1 else None}
            print(f"[shard_scaling] {mp} N={n} max {tmax:.4f}s max/mean {per_n[n]['balance_max_over_mean']}",
                  file=sys.stderr, flush=True)
        out["per_map"][mp] = per_n
    print(json.dumps(out))


if __name__ == "__main__":
    main()

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

import numpy as np
import os
import sys
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]


def learned_table(ds, params, n):
    """The cost table an N-rank job learns from its first gathered frame: each shard rendered once (probe plan) in
    its own workspace, its measured per-shard-tile costs placed at their frame tiles through the deal order."""
    n_tiles = -(-params.width // params.tile_w) * -(-params.height // params.tile_h)
    table = np.zeros((2, n_tiles), dtype=np.uint32)
    for s in range(n):
        sp = replace(params, shard=s, num_shards=n)
        w = ds.workspace()
        ds.reserve(sp, w)
        ds.render_device_sync(sp, w) if hasattr(ds, "render_device_sync") else _render_ws(ds, sp, w)
        order = ds.tile_map(sp, w)
        c = ds.tile_costs(sp, w)
        tiles = order[s::n][:c.shape[1]]
        table[:, tiles] = c
        w.close()
    return table


def _render_ws(ds, sp, w):
    import torch
    from rtpotato.scene import shard_slot_count
    out = torch.zeros(3 * max(1, shard_slot_count(sp)), dtype=torch.float64, device="cuda")
    ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    ds.render_device(sp, out, ctr, workspace=w)
    torch.cuda.synchronize()


def inflight_time(ds, sp, F, frames, table=None, per_launch=1, order="interleaved"):
    """Steady per-frame time of shard sp with F launches in flight (bench.py's loop without the gather): launches of
    per_launch frames (rp_render_frames_device_ws, interleaved) alternate over F streams and workspaces; one warm-up
    round, then `frames` frames (in launches of per_launch) timed together."""
    import time
    import torch
    from rtpotato.scene import shard_slot_count
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    wss = [ds.workspace() for _ in range(F)]
    L = per_launch
    for w in wss:
        ds.reserve_frames(sp, L, w)
        if table is not None:
            ds.set_tile_costs(sp, table, sp.num_shards, w)
    n = shard_slot_count(sp)
    bufs = [torch.zeros(3 * max(1, n) * L, dtype=torch.float64, device=dev) for _ in range(F)]
    ctrs = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(F)]

    def launch(i):
        if L == 1:
            ds.render_device(sp, bufs[i], ctrs[i], stream=streams[i], workspace=wss[i])
        else:
            ds.render_frames_device(sp, L, bufs[i], ctrs[i], stream=streams[i], workspace=wss[i], order=order)

    for i in range(F):
        launch(i)
    torch.cuda.synchronize()
    launches = max(1, frames // L)
    t0 = time.perf_counter()
    for k in range(launches):
        launch(k % F)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (launches * L)
    rays = int(ctrs[0][0]) // L
    assert all(int(c[3]) == 0 for c in ctrs)
    for w in wss:
        w.close()
    return dt, rays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--tile", type=int, default=0, help="square tile size (default: the config's)")
    ap.add_argument("--maps", default="interleave,balanced")
    ap.add_argument("--reps", type=int, default=3, help="renders per shard; the shard's time is their median")
    ap.add_argument("--inflight", type=int, default=1,
                    help="frames in flight (> 1: each shard renders --frames frames on this many streams and "
                         "workspaces, as bench.py does for N > 1; its time is the steady per-frame time)")
    ap.add_argument("--frames", type=int, default=9)
    ap.add_argument("--per-launch", type=int, default=1,
                    help="frames per launch (> 1: rp_render_frames_device_ws, interleaved, as bench.py renders them)")
    ap.add_argument("--learned", type=int, default=1,
                    help="1: schedule balanced N > 1 shards from a learned cost table (what every rank holds after "
                         "its first gathered frame: the measured costs of all shards, combined through the deal order "
                         "and installed with rp_workspace_set_tile_costs); 0: the whole-frame probe every frame")
    ap.add_argument("--opt", action="append", default=[], help="rp_scene_options field=value (as bench.py --opt)")
    ap.add_argument("--frame-order", default="pixel", choices=("interleaved", "pixel"),
                    help="RP_FRAME_ORDER_* of a launch of several frames (bench.py's default: pixel)")
    a = ap.parse_args()
    options = {}
    for kv in a.opt:
        k, v = kv.split("=", 1)
        options[k] = float(v) if k == "cost_traverse" else (
            v if k in ("builder", "engine", "node_format", "tile_order", "unit_queues", "collapse", "node_layout") else int(v))
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    scene, params = scenes.config_scene(a.config)
    if a.tile:
        params = replace(params, tile_w=a.tile, tile_h=a.tile)
    ds = DeviceScene(scene, options=options)
    ds.render(replace(params, spp=4))  # warm
    out = {"config": a.config, "tile": [params.tile_w, params.tile_h], "reps": a.reps, "inflight": a.inflight,
           "per_launch": a.per_launch, "frame_order": a.frame_order,
           "scene_options": options or "defaults", "per_map": {}}
    import statistics
    for mp in a.maps.split(","):
        smap = {"interleave": 0, "balanced": 1}[mp]
        per_n, t1 = {}, None
        for n in [int(x) for x in a.ns.split(",")]:
            times, rays = [], 0
            table = learned_table(ds, replace(params, shard_map=smap), n) if a.learned and n > 1 and smap else None
            for s in range(n):
                sp = replace(params, shard=s, num_shards=n, shard_map=smap)
                if table is not None:
                    ds.set_tile_costs(sp, table, n)
                if a.inflight > 1 or a.per_launch > 1:
                    t, r = inflight_time(ds, sp, a.inflight, a.frames, table, a.per_launch, a.frame_order)
                    times.append(t)
                    rays += r
                    continue
                reps = []
                for _ in range(a.reps):
                    _, _, st = ds.render(sp)
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

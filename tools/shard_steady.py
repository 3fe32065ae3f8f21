"""Steady-state ray rate of a shard against the whole frame, tails removed.

Each case renders `--per-launch` frames in one persistent launch (rp_render_frames_device_ws), so a launch's tail is
spread over many frames, and reports Mrays/s.  Cases, all of `--config`'s scene (names are C3's spp):
  frame_256spp        the whole frame (the N = 1 work)
  frame_32spp         the whole frame at 1/8 of the samples -- a shard's ray count over all the frame's tiles
  shard_balanced      shard 3 of 8, balanced deal by the learned cost table (bench.py's N = 8 per-rank work)
  shard_interleave    shard 3 of 8, tiles t with t % 8 = 3
  shard_morton        shard 3 of 8, balanced deal of Z-order square blocks (tile_order = morton)
Tells whether an 8-way shard's per-ray cost comes from the number of units (frame_32spp slow too) or from which
tiles it holds (only the shards slow).  A case may carry modifiers, `name:spp=..:sps=..:tile=..:L=..:opt.<field>=..`
(e.g. `frame_256spp:opt.tile_order=plain`, `shard_balanced:tile=16`, `shard_balanced:order=sequential`).

    python tools/shard_steady.py --per-launch 16 --reps 2
"""
import argparse
import json
import os
import sys
import time
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd"), os.path.join(REPO, "tools")]


def rate(ds, sp, L, launches, table, order="auto"):
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    dev = torch.device("cuda", 0)
    n = max(1, shard_slot_count(sp))
    w = ds.workspace()
    ds.reserve_frames(sp, L, w)
    if table is not None:
        ds.set_tile_costs(sp, table, sp.num_shards, w)
    buf = torch.zeros(3 * n * L, dtype=torch.float64, device=dev)
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
    ds.render_frames_device(sp, L, buf, ctr, workspace=w, order=order)  # warm-up (learns costs when the shard is the frame)
    torch.cuda.synchronize()
    rays = 0
    t0 = time.perf_counter()
    for _ in range(launches):
        ds.render_frames_device(sp, L, buf, ctr, workspace=w, order=order)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rays = int(ctr[0]) * launches
    assert int(ctr[3]) == 0
    w.close()
    return {"ms_per_frame": round(dt * 1e3 / (launches * L), 3), "mrays_per_s": round(rays / dt / 1e6, 1),
            "rays_per_frame": int(ctr[0]) // L}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--per-launch", type=int, default=16)
    ap.add_argument("--launches", type=int, default=2)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--cases", default="frame_256spp,frame_32spp,shard_balanced,shard_interleave,shard_morton")
    a = ap.parse_args()
    import torch  # noqa: F401
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    from shard_scaling import learned_table
    scene, params = scenes.config_scene(a.config)
    out = {"config": a.config, "per_launch": a.per_launch, "launches": a.launches, "runs": {}}
    dss = {}

    def scene_for(opt):
        key = json.dumps(opt, sort_keys=True)
        if key not in dss:
            ds = DeviceScene(scene, options=opt or None)
            ds.render(replace(params, spp=4))
            dss[key] = ds
        return dss[key]

    tables = {}
    for rep in range(a.reps):
        for case in a.cases.split(","):
            base, *mods = case.split(":")
            opt, table, L, sp, order = {}, None, a.per_launch, params, "auto"
            for m in mods:  # modifiers: spp=, sps=, tile=, L=, opt.<field>=
                k, v = m.split("=", 1)
                if k == "spp":
                    sp = replace(sp, spp=int(v))
                elif k == "sps":
                    sp = replace(sp, samples_per_stream=int(v))
                elif k == "tile":
                    sp = replace(sp, tile_w=int(v), tile_h=int(v))
                elif k == "L":
                    L = int(v)
                elif k == "order":
                    order = v
                elif k.startswith("opt."):
                    opt[k[4:]] = v if not v.isdigit() else int(v)
            if base == "frame_256spp":
                L = L if any(m.startswith("L=") for m in mods) else max(1, a.per_launch // 8)
            elif base == "frame_32spp":
                sp = replace(sp, spp=32)
            else:
                smap = 0 if base == "shard_interleave" else 1
                if base == "shard_morton":
                    opt["tile_order"] = "morton"
                full = replace(sp, shard_map=smap)
                sp = replace(full, shard=3, num_shards=8)
                if smap:
                    tk = json.dumps([case, opt], sort_keys=True)
                    if tk not in tables:
                        tables[tk] = learned_table(scene_for(opt), full, 8)
                    table = tables[tk]
            r = rate(scene_for(opt), sp, L, a.launches, table, order)
            r["frames_per_launch"] = L
            out["runs"].setdefault(case, []).append(r)
            print(f"rep {rep} {case}: {r}", file=sys.stderr, flush=True)
    out["best_mrays_per_s"] = {k: max(r["mrays_per_s"] for r in v) for k, v in out["runs"].items()}
    base = out["best_mrays_per_s"].get("frame_256spp")
    if base:
        out["rate_over_frame_256spp"] = {k: round(v / base, 4) for k, v in out["best_mrays_per_s"].items()}
    for ds in dss.values():
        ds.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

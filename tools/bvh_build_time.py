"""Setup and traversal of the two acceleration-structure builders on config C5's scene (10 M random
triangles): rp_scene_create time with the host binned SAH and with the device LBVH, tree statistics, and
a 4-spp C5 frame over each tree.  Diagnostic only.

    python tools/bvh_build_time.py [--tris 10000000] [--spp 4] [--builders gpu,host:q8,host@2:f32,...]
"""
import argparse
import json
import os
import sys
import time
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--builders", default="gpu,host")
    a = ap.parse_args()
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    t = time.time()
    from rtpotato.scene import RenderParams
    cfg = scenes.CONFIGS["C5"]
    sc = scenes.configure(scenes.random_mesh(a.tris), cfg.width, cfg.height)
    params = RenderParams(cfg.width, cfg.height, a.spp, 8, scenes.DEFAULT_SEED)
    out = {"tris": a.tris, "spp": a.spp, "mesh_seconds": round(time.time() - t, 2)}
    DeviceScene(scenes.configure(scenes.random_mesh(1000), 64, 64)).close()  # HIP runtime + code objects
    print(f"[bvh] mesh ready {out['mesh_seconds']}s", file=sys.stderr, flush=True)
    for spec in a.builders.split(","):
        spec_, _, fmt = spec.partition(":")  # builder[@max_leaf][:node_format]
        b, _, leaf = spec_.partition("@")
        opt = {"builder": b}
        if leaf:
            opt["max_leaf"] = int(leaf)
        if fmt:
            opt["node_format"] = fmt
        t = time.time()
        ds = DeviceScene(sc, options=opt)
        setup = time.time() - t
        info = ds.info()
        ds.render(replace(params, spp=1, width=256, height=256))
        _, _, st = ds.render(params)
        out[spec] = {"scene_create_s": round(setup, 3), "phases_s": ds.build_times(), "info": info, "frame_s": round(st["seconds"], 4),
                  "mrays_s": round(st["rays"] / st["seconds"] / 1e6, 1), "rays": st["rays"]}
        print(f"[bvh] {spec}: {out[spec]}", file=sys.stderr, flush=True)
        ds.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Per-ray event counts of the reference traversal (reference median-split tree, reference visit order),
measured by the CPU oracle's instrumented restatement at each config's fixed seed.  bench.py turns them
into algorithmic bytes / flops per ray for the roofline.  Test infrastructure output.

    python tests/golden/make_event_counts.py   ->   tests/golden/event_counts.json

Sample per config: every 64th 32x32 tile (shard 5 of 64) of the full-size frame at the config's spp
(C1: the whole 320x180x4 frame; C5: every 1024th tile from the centre column at 4 spp); per-unit seeding makes the sample a subset
of the real frame.
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]

from oracle import oracle_py as O  # noqa: E402
from rtpotato import scenes  # noqa: E402
from rtpotato.scene import RenderParams  # noqa: E402


def main():
    out = {}
    for name in ("C1", "C2", "C3", "C5"):
        scene, params = scenes.config_scene(name)
        if name == "C5":  # 10M triangles: 16 of the 16,384 tiles (the centre column) at 4 spp
            params = RenderParams(params.width, params.height, 4, 8, params.seed, 32, 32, 64, 1024)  # centre column
        elif name != "C1":
            params = RenderParams(params.width, params.height, params.spp, 8, params.seed, 32, 32, 5, 64)
        d = scene.desc()
        os_ = O.OracleScene(d.addr(), d)
        cam, p = scene.camera.to_c(), params.to_c()
        t = time.time()
        _, _, c = os_.render(ctypes.addressof(cam), ctypes.addressof(p), params.width, params.height,
                             threads=os.cpu_count() or 8)
        rays = c["rays"]
        out[name] = {"sample": f"{params.width}x{params.height}x{params.spp} shard {params.shard}/{params.num_shards}",
                     "rays": rays, "samples": c["samples"],
                     "per_ray": {k: c[k] / rays for k in ("box_tests", "tri_tests", "sphere_tests", "tri_hits", "texels")},
                     "rays_per_sample": rays / c["samples"]}
        print(name, round(time.time() - t, 1), "s", out[name])
    json.dump(out, open(os.path.join(HERE, "event_counts.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

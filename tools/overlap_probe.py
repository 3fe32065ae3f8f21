"""Frames in flight: K consecutive frames of one shard rendered back to back on one stream (one
workspace) against the same K frames alternating over two streams with two workspaces (two device
scenes of the same scene), so one frame's tail overlaps the next frame's start.  Diagnostic only.

    python tools/overlap_probe.py [--config C3] [--shards 1,8] [--frames 6]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--shards", default="1,8")
    ap.add_argument("--frames", type=int, default=6)
    a = ap.parse_args()
    import torch
    from dataclasses import replace
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    from rtpotato.scene import shard_slot_count
    scene, params = scenes.config_scene(a.config)
    dss = [DeviceScene(scene), DeviceScene(scene)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    out = {"config": a.config, "frames": a.frames, "per_n": {}}
    for n in [int(x) for x in a.shards.split(",")]:
        p = replace(params, shard=0, num_shards=n)
        m = shard_slot_count(p)
        bufs = [torch.zeros(3 * m, dtype=torch.float64, device="cuda") for _ in range(2)]
        ctrs = [torch.zeros(4, dtype=torch.int64, device="cuda") for _ in range(2)]
        for ds in dss:
            ds.reserve(p)
        res = {}
        for mode in ("serial", "two_streams", "serial", "two_streams"):
            k2 = 2 if mode == "two_streams" else 1
            for i in range(2):  # warm both workspaces
                dss[i].render_device(p, bufs[i], ctrs[i], stream=streams[i])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in range(a.frames):
                i = f % k2
                dss[i].render_device(p, bufs[i], ctrs[i], stream=streams[i])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.frames
            res.setdefault(mode, []).append(round(dt * 1e3, 3))
        same = bool(torch.equal(bufs[0], bufs[1]))
        out["per_n"][n] = {"ms_per_frame": res, "frames_identical": same}
        print(f"[overlap] N={n} {res}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

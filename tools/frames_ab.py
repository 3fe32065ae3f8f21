"""Several frames per persistent launch against one frame per launch (rp_render_frames_device_ws).

A frame's tail -- the last units of a launch, run by a few sparse waves while most of the GPU idles -- costs C3 ~4 % of
its frame on one GPU and an 8-way shard ~20 % (profiles/r5/c3_shard_overhead_counters.json).  With L frames per launch
the lanes frame f's tail leaves take frame f + 1's units; only the launch's last frame has a tail.  This tool times,
on one GPU, `--frames` frames of a config (or of one shard of its balanced N-way deal, with the learned cost table an
N-rank job installs after its first gathered frame) rendered

  - one per launch, sequentially (bench.py's N = 1 loop),
  - one per launch, `--inflight` launches in flight on their own streams and workspaces (bench.py's N > 1 loop),
  - L per launch, for each L of `--per-launch`,

and reports ms per frame and the launches' kernel durations (HIP events).  Frames differ by seed only (frame f of a
launch = the frame of seed + f * B * W * H), so every mode renders the same amount of work per frame up to noise.

    python tools/frames_ab.py --config C3 --frames 8 --per-launch 2,4,8
    python tools/frames_ab.py --config C3 --shard-of 8 --shard 3 --frames 32 --per-launch 4,8,16
"""
import argparse
import json
import os
import sys
import time
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd"), os.path.join(REPO, "tools")]


def timed(ds, sp, frames, per_launch, inflight, table):
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    dev = torch.device("cuda", 0)
    n = max(1, shard_slot_count(sp))
    streams = [torch.cuda.current_stream(dev)] if inflight == 1 else [torch.cuda.Stream(dev) for _ in range(inflight)]
    wss = [ds.workspace() for _ in range(inflight)]
    for w in wss:
        ds.reserve_frames(sp, per_launch, w)
        if table is not None:
            ds.set_tile_costs(sp, table, sp.num_shards, w)
    bufs = [torch.zeros(3 * n * per_launch, dtype=torch.float64, device=dev) for _ in range(inflight)]
    ctrs = [torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev) for _ in range(inflight)]
    launches = frames // per_launch
    stride = (-(-sp.spp // (sp.samples_per_stream or F.RP_SAMPLES_PER_STREAM))) * sp.width * sp.height

    def launch(k, ev=None):
        i = k % inflight
        q = replace(sp, seed=sp.seed + k * per_launch * stride)
        if ev:
            ev[0].record(streams[i])
        if per_launch == 1:
            ds.render_device(q, bufs[i], ctrs[i], stream=streams[i], workspace=wss[i])
        else:
            ds.render_frames_device(q, per_launch, bufs[i], ctrs[i], stream=streams[i], workspace=wss[i])
        if ev:
            ev[1].record(streams[i])

    for k in range(inflight):  # warm-up: every workspace learns its costs (whole frames on one device)
        launch(k)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    t0 = time.perf_counter()
    for k in range(launches):
        launch(k, evs[k])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rays = sum(int(c[0]) for c in ctrs)
    assert all(int(c[3]) == 0 for c in ctrs)
    for w in wss:
        w.close()
    kms = [s.elapsed_time(e) for s, e in evs]
    return {"ms_per_frame": round(dt * 1e3 / (launches * per_launch), 3), "launches": launches,
            "kernel_ms_mean": round(sum(kms) / len(kms), 3), "kernel_ms_per_frame": round(sum(kms) / len(kms) / per_launch, 3),
            "rays_per_frame_last": rays // (inflight * per_launch)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--per-launch", default="2,4,8")
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--shard-of", type=int, default=1)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--samples-per-stream", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch  # noqa: F401
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    from shard_scaling import learned_table
    scene, params = scenes.config_scene(a.config)
    if a.samples_per_stream:
        params = replace(params, samples_per_stream=a.samples_per_stream)
    ds = DeviceScene(scene)
    ds.render(replace(params, spp=4))
    table = None
    if a.shard_of > 1:
        params = replace(params, shard_map=1)
        table = learned_table(ds, params, a.shard_of)
    sp = replace(params, shard=a.shard, num_shards=a.shard_of)
    out = {"config": a.config, "samples_per_stream": params.samples_per_stream or 32, "frames": a.frames,
           "shard": f"{a.shard} of {a.shard_of}" + (" (balanced, learned table)" if a.shard_of > 1 else ""),
           "runs": {}}
    modes = [("one_per_launch", 1, 1), (f"one_per_launch_{a.inflight}_inflight", 1, a.inflight)]
    modes += [(f"{L}_per_launch", L, 1) for L in (int(x) for x in a.per_launch.split(","))]
    for rep in range(a.reps):
        for name, L, inf in modes:
            r = timed(ds, sp, a.frames, L, inf, table)
            out["runs"].setdefault(name, []).append(r)
            print(f"rep {rep} {name}: {r}", file=sys.stderr, flush=True)
    base = min(r["ms_per_frame"] for r in out["runs"]["one_per_launch"])
    out["best_ms_per_frame"] = {k: min(r["ms_per_frame"] for r in v) for k, v in out["runs"].items()}
    out["speedup_vs_one_per_launch"] = {k: round(base / v, 4) for k, v in out["best_ms_per_frame"].items()}
    ds.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

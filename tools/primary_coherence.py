"""Ceiling of a coherent primary-ray pass: how much faster camera rays traverse when a wave holds
64 neighbouring camera rays instead of 64 unrelated ones.

With lens_radius = 0 a camera ray's direction depends only on its jitter words (render.rs:36-44: the UnitDisk sample is
multiplied by 0; render.rs:74-82: the jitter comes from a clone of the stream), so a frame's primary hits could be
traced ahead of the path loop in any order.  This tool times rp_intersect (intersect_kernel: one ray per lane, the
product traversal and exact f64 tests, plus the full hit record) over the same N camera rays of a config's frame in
three orders:
  coherent  -- 2 x 2 pixels x 16 jittered samples per 64 consecutive rays, quads in tile order (a wave = one quad);
  pixels    -- 64 neighbouring pixels (8 x 8) with one sample each per wave, tiles in order;
  shuffled  -- a random permutation (the megakernel's view: a wave's lanes are at unrelated units and bounces).
The kernel durations come from the rocprofv3 kernel trace of this run (--trace DIR) or from HIP events around the
call's kernel (the ctypes call also copies the rays and hits over PCIe; those copies are outside the kernel trace).

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/primary_coherence.py --config C5
    python3 tools/primary_coherence.py --config C5 --trace OUT    # summarise a finished trace
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]

ORDERS = ("coherent", "pixels", "shuffled")


def camera_rays(scene, W, H, n, seed=1):
    """n camera rays of a W x H frame (lens 0): render.rs:32-52 in numpy, f64, same operation order as start_sample
    (rp_device.h).  Returns (rays (n, 8) in `coherent` order, the pixel of each ray)."""
    cam = scene.camera
    assert cam.lens_radius == 0.0, "the coherent pass applies to lens_radius = 0 only"
    m = np.array(cam.transformation.orientation, dtype=np.float64)  # column-major
    pos = np.array(cam.transformation.position, dtype=np.float64)
    tanf = np.tan(0.5 * cam.fov)
    focal, aspect = cam.focal_dist, cam.aspect_ratio
    rng = np.random.default_rng(seed)
    # quads of 2 x 2 pixels in tile order (32 x 32 tiles, row-major quads inside), 16 samples per pixel; enough quads
    quads_needed = -(-n // 64)
    tiles_x, tiles_y = -(-W // 32), -(-H // 32)
    # sample the frame evenly, whole tiles: every k-th tile of the frame, all of its quads
    qx, qy = np.meshgrid(np.arange(16), np.arange(16))
    tq = np.stack([qx.ravel(), qy.ravel()], 1)  # 256 quads per tile, row-major
    tiles = [(tx, ty) for ty in range(tiles_y) for tx in range(tiles_x)]
    step = max(1, len(tiles) * 256 // quads_needed)
    quads = np.concatenate([tq + np.array([tx * 16, ty * 16]) for tx, ty in tiles[::step]])
    quads = quads[(quads[:, 0] * 2 < W) & (quads[:, 1] * 2 < H)][:quads_needed]
    px = np.empty((len(quads), 64, 2), dtype=np.int64)
    lane = np.arange(64)
    px[:, :, 0] = quads[:, None, 0] * 2 + (lane // 16) % 2
    px[:, :, 1] = quads[:, None, 1] * 2 + (lane // 32)
    px = np.minimum(px.reshape(-1, 2)[:n], [W - 1, H - 1])
    ju = (px[:, 0] + rng.random(len(px))) / W
    jv = (px[:, 1] + rng.random(len(px))) / H
    x = (2.0 * ju - 1.0) * tanf * focal * aspect
    y = (2.0 * jv - 1.0) * tanf * focal
    z = np.full_like(x, -focal)
    nrm = np.sqrt((x * x + y * y) + z * z)
    dl = np.stack([x / nrm, y / nrm, z / nrm], 1)
    d = np.stack([(dl[:, 0] * m[0] + dl[:, 1] * m[3]) + dl[:, 2] * m[6],
                  (dl[:, 0] * m[1] + dl[:, 1] * m[4]) + dl[:, 2] * m[7],
                  (dl[:, 0] * m[2] + dl[:, 1] * m[5]) + dl[:, 2] * m[8]], 1)
    rays = np.empty((len(px), 8), dtype=np.float64)
    rays[:, 0:3] = pos
    rays[:, 3:6] = d
    rays[:, 6] = 1e-3  # RAY_EPSILON: Camera rays are traced from t_min = RAY_EPSILON (render.rs:105)
    rays[:, 7] = np.inf
    return rays, px


def pixel_order(px, W):
    """8 x 8 pixel blocks with one sample per pixel per wave: sort by (8x8 block in tile order, sample rank, pixel)."""
    bx, by = px[:, 0] // 8, px[:, 1] // 8
    tile = (px[:, 1] // 32) * (-(-W // 32)) + px[:, 0] // 32
    blk = (by % 4) * 4 + bx % 4
    pix = (px[:, 1] % 8) * 8 + px[:, 0] % 8
    # rank of the sample within its pixel: in the coherent order lanes 16p..16p+15 of a quad are pixel p's samples
    rank = np.arange(len(px)) % 16
    return np.lexsort((pix, rank, blk, tile))


def summarise(trace_dir, meta):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "intersect_kernel" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    runs = meta["runs"]
    assert len(rows) == len(runs), (len(rows), len(runs))
    out = {}
    for (t0, dur), name in zip(rows, runs):
        out.setdefault(name, []).append(dur / 1e6)
    n = meta["n"]
    res = {k: {"ms": [round(x, 3) for x in v], "grays_per_s": round(n / (min(v) / 1e3) / 1e9, 3)} for k, v in out.items()}
    res["coherent_over_shuffled"] = round(min(out["shuffled"]) / min(out["coherent"]), 3)
    res["pixels_over_shuffled"] = round(min(out["shuffled"]) / min(out["pixels"]), 3)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--n", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--trace", default="", help="summarise this rocprofv3 kernel-trace directory (no rendering)")
    ap.add_argument("--meta", default="gpurun_out/primary_coherence_meta.json")
    args = ap.parse_args()
    if args.trace:
        meta = json.load(open(args.meta))
        meta["kernel_times"] = summarise(args.trace, meta)
        print(json.dumps(meta, indent=1))
        return
    import torch  # noqa: F401  (librp shares torch's HIP runtime)
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    scene, params = scenes.config_scene(args.config)
    ds = DeviceScene(scene, device=0)
    rays, px = camera_rays(scene, params.width, params.height, args.n)
    n = len(rays)
    perm = {"coherent": np.arange(n), "pixels": pixel_order(px, params.width),
            "shuffled": np.random.default_rng(7).permutation(n)}
    runs = []
    ref = None
    for rep in range(args.reps):
        for name in ORDERS:
            p = perm[name]
            hits, mats = ds.intersect(rays[p])
            inv = np.empty(n, dtype=np.int64)
            inv[p] = np.arange(n)
            t = hits[inv, 0]
            if ref is None:
                ref = t
            assert np.array_equal(t, ref), name  # the same closest hits in every order
            runs.append(name)
            print(f"{name} rep {rep}: {np.isfinite(t).mean():.3f} of rays hit", file=sys.stderr, flush=True)
    meta = {"config": args.config, "n": n, "runs": runs, "hit_fraction": float(np.isfinite(ref).mean()),
            "frame": [params.width, params.height], "scene_info": ds.info()}
    os.makedirs(os.path.dirname(args.meta) or ".", exist_ok=True)
    json.dump(meta, open(args.meta, "w"), indent=1, default=str)
    ds.close()


if __name__ == "__main__":
    main()

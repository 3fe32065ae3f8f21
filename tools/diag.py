"""Diagnostic run (not a benchmark): phase breakdown of the render kernel from the RPK_DIAG build.

    RP_LIB=raytracing-potato_amd/lib/librp_diag.so python tools/diag.py [--config C3] [--spp 32]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--shards", type=int, default=1, help="render shard --shard of N (per-rank work of an N-GPU run)")
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--balanced", action="store_true", help="the balanced tile plan (RP_SHARD_BALANCED), learned from a "
                                                            "whole-frame render of every shard first (tools/shard_scaling.py)")
    ap.add_argument("--sps", type=int, default=0, help="samples_per_stream (the RNG contract; 0 = 32, >= spp: one "
                                                       "stream per pixel)")
    ap.add_argument("--opt", action="append", default=[], help="rp_scene_options field=value")
    ap.add_argument("--frames", type=int, default=1,
                    help="> 1: one launch of this many frames (rp_render_frames_device_ws, bench.py's loop), measured "
                         "after a warm launch of the same size on the same workspace; the timeline bins (10 ms, 64 of "
                         "them) then cover only the launch's first 640 ms")
    ap.add_argument("--frame-order", default="pixel", choices=("interleaved", "pixel", "sequential"))
    a = ap.parse_args()
    os.environ.setdefault("RP_LIB", os.path.join(REPO, "raytracing-potato_amd", "lib", "librp_diag.so"))
    from dataclasses import replace
    from rtpotato import _ffi as F, scenes
    from rtpotato.render import DeviceScene
    scene, params = scenes.config_scene(a.config)
    params = replace(params, spp=a.spp, shard=a.shard, num_shards=a.shards, samples_per_stream=a.sps,
                     shard_map=1 if a.balanced else 0)
    opts = {}
    for kv in a.opt:
        k, v = kv.split("=", 1)
        opts[k] = float(v) if k == "cost_traverse" else (v if not v.lstrip("-").isdigit() else int(v))
    ds = DeviceScene(scene, options=opts)
    ds.render(replace(params, spp=1))  # warm
    if a.balanced and a.shards > 1:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from shard_scaling import learned_table
        ds.set_tile_costs(params, learned_table(ds, params, a.shards), a.shards)
    NDIAG = 416  # rp_kernel.h DIAG_N
    buf = (ctypes.c_uint64 * NDIAG)()
    if a.frames > 1:
        import time
        import torch
        from rtpotato.scene import shard_slot_count
        ds.reserve_frames(params, a.frames)
        n = shard_slot_count(params)
        out_rgb = torch.zeros(a.frames * 3 * max(1, n), dtype=torch.float64, device="cuda")
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        ds.render_frames_device(params, a.frames, out_rgb, ctr, order=a.frame_order)  # warm: learns the tile costs
        torch.cuda.synchronize()
        ctr.zero_()
        F.check(F.rp().rp_diagnostics(ds.handle, buf, NDIAG, 1))
        t = time.perf_counter()
        ds.render_frames_device(params, a.frames, out_rgb, ctr, order=a.frame_order)
        torch.cuda.synchronize()
        st = {"rays": int(ctr[0]), "seconds": time.perf_counter() - t}
        assert int(ctr[3]) == 0, "status bits set"
    else:
        F.check(F.rp().rp_diagnostics(ds.handle, buf, NDIAG, 1))
        _, _, st = ds.render(params)
    F.check(F.rp().rp_diagnostics(ds.handle, buf, NDIAG, 1))
    d = list(buf)
    ph = d[:5]
    tot = sum(ph)
    iters, active, trips, visits, tests = d[5], d[6], d[7], d[8], d[9]
    out = {
        "config": a.config, "spp": a.spp, "samples_per_stream": a.sps or 32, "rays": st["rays"], "seconds": st["seconds"],
        "frames_per_launch": a.frames, **({"frame_order": a.frame_order} if a.frames > 1 else {}),
        "phase_share": {k: round(v / tot, 4) for k, v in zip(["fetch", "rng_refill", "traverse", "shade", "tail"], ph)},
        "wave_iterations": iters, "lanes_active_at_traverse": round(active / max(1, iters) / 64, 4),
        "visits_per_ray": round(visits / st["rays"], 3), "prim_tests_per_ray": round(tests / st["rays"], 3),
        "traversal_lane_util": round(visits / max(1, trips * 64), 4),
        "trips_per_wave_iteration": round(trips / max(1, iters), 2),
        "wave_cycles_per_iteration": round(tot / max(1, iters), 1),
        "traverse_cycles_per_trip": round(ph[2] / max(1, trips), 1),
    }
    slow = {"ticks": d[13] >> 32, "ms": round((d[13] >> 32) / 1e5, 3), "pixel": [d[13] & 0xFFFF, (d[13] >> 16) & 0xFFF],
            "batch": (d[13] >> 28) & 0xF, "rays": d[14] & 0xFFFFFFFF}
    t0, tq, t1 = (~d[10]) & (2**64 - 1), (~d[11]) & (2**64 - 1), d[12]
    if t1 > t0:  # 100 MHz real-time clock
        out["slowest_unit"] = slow
        out["timeline_ms"] = {"queue_drained": round((tq - t0) / 1e5, 3), "last_exit": round((t1 - t0) / 1e5, 3),
                              "tail_frac": round((t1 - tq) / (t1 - t0), 4)}
    regions = ["node", "prim", "step", "shade", "surface", "sph_uv", "texture", "lambert", "metal", "dielectric",
               "loop_lambert", "loop_metal", "end_sample", "end_pixel", "start_sample", "refill", "rng_fallback",
               "jit_fallback", "begin_pixel", "ring_load", "round", "miss"]
    out["regions"] = {
        name: {"wave_execs_per_kray": round(1000 * d[16 + 2 * i] / st["rays"], 2),
               "lane_util": round(d[17 + 2 * i] / max(1, 64 * d[16 + 2 * i]), 3)}
        for i, name in enumerate(regions)}
    cyc = ["surface", "sph_uv", "tex_issue", "scatter", "tex_value", "emit_accum", "start_sample", "end_sample",
           "newray_always", "refill", "next_bounce", "node_loop", "prim_loop"]
    out["cycle_share"] = {name: round(d[320 + i] / tot, 4) for i, name in enumerate(cyc)}
    # Loss budget: per cycle region, the share of all wave-cycles its idle lanes cost, cycle share x
    # (1 - lane utilisation of the region's DREG counter).  Scatter pools the per-material regions and their rejection
    # loops (lanes summed over execs); emission/accumulation takes the shade region's utilisation.
    reg = {name: (d[16 + 2 * i], d[17 + 2 * i]) for i, name in enumerate(regions)}
    def util(*names):
        e = sum(reg[n][0] for n in names)
        return reg_l / (64 * e) if (e and (reg_l := sum(reg[n][1] for n in names))) else None
    umap = {"node_loop": ("node",), "prim_loop": ("prim",), "surface": ("surface",), "sph_uv": ("sph_uv",),
            "tex_issue": ("texture",), "tex_value": ("texture",),
            "scatter": ("lambert", "metal", "dielectric", "loop_lambert", "loop_metal"), "emit_accum": ("shade",),
            "start_sample": ("start_sample",), "end_sample": ("end_sample",), "refill": ("refill",)}
    lb = {}
    for name, names in umap.items():
        u = util(*names)
        share = d[320 + cyc.index(name)] / tot
        lb[name] = {"cycle_share": round(share, 4), "lane_util": round(u, 3) if u is not None else None,
                    "idle_share": round(share * (1 - u), 4) if u is not None else None}
    named = sum(d[320 + i] for i in range(len(cyc))) / tot
    out["loss_budget"] = {"regions": dict(sorted(lb.items(), key=lambda kv: -(kv[1]["idle_share"] or 0))),
                          "idle_share_total": round(sum(v["idle_share"] or 0 for v in lb.values()), 4),
                          "named_cycle_share": round(named, 4),
                          "note": "share of all wave-cycles spent in each region x (1 - its lane utilisation): the "
                                  "issue slots idle lanes cost; the rest of the wave-cycles (1 - named_cycle_share) is "
                                  "the round's control (ballots, ray setup, queue fetch)"}
    # timeline histograms (10 ms bins from each block's start): lanes retiring, pixels fetched and their rays
    last = max([b for b in range(64) if d[64 + b] or d[192 + b]] or [0])
    out["timeline_10ms"] = [{"t_ms": 10 * b, "retired_lanes": d[64 + b], "pixels": d[192 + b],
                             "rays_per_pixel": round(d[128 + b] / max(1, d[192 + b]), 1),
                             "max_rays_unit": d[256 + b]} for b in range(last + 1)]
    # unit durations (rp_kernel.h DIAG_DUR): log2 bins of 100 MHz ticks from 2^10 (10.24 us)
    out["unit_durations"] = [{"ms_from": round(2 ** (10 + b) / 1e5, 3), "ms_to": round(2 ** (11 + b) / 1e5, 3),
                              "units": d[352 + b], "rays_per_unit": round(d[376 + b] / max(1, d[352 + b]), 1)}
                             for b in range(24) if d[352 + b]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

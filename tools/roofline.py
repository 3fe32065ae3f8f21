"""Per-ray roofline record of the frame kernel from rocprofv3 --pmc passes over one bench frame.

    python tools/roofline.py --config C3 --bench BENCH.json --out OUT.json PASS_DIR [PASS_DIR ...]

Each PASS_DIR is the -d directory of one `rocprofv3 --pmc ... -- python3 bench.py --steps 8 --warmup 0`
run (one dispatch of the frame kernel per run, rendering its frames_per_launch frames); BENCH.json is that bench's
stdout line (its rays per frame and frames per launch).
The record bench.py prices its `roofline` with (kernel_record()): per ray of the frame kernel
  - traffic_bytes_per_ray: memory-side bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; FETCH_SIZE doubled,
    the gfx950 correction of MI355X_MICROARCH.md "HBM"; Infinity-Cache hits are counted, so this is an upper
    bound of HBM traffic),
  - valu_per_ray / salu_per_ray / vmem_per_ray / lds_per_ray: wave-instructions,
and for the frame: the SQ cycle budget (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES, all in
quad-cycles), the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration), the VALU-issue fraction at
that clock and at 2.4 GHz (a wave64 VALU instruction holds a SIMD-32 for 2 cycles), and the instruction mix.

With --diag (a tools/diag.py record of the same build over the same frame) the record also carries the kernel's
own ALGORITHMIC bytes per ray -- what its traversal and shading must touch, wherever it is served from:
  node visits x bytes a visit loads (Node4 f32: 6 plane rows + children = 112 B; Node4Q: 64 B)
  + primitive tests x 80 B (rpl::Prim)
  + shaded hits x 232 B (PrimRef 16 + 3 vertex normals 72 + 3 vertex uvs 48 + Material 96)
  + texture samples x 4 B (one RGBA8 texel)
  + keystream blocks made x 128 B (64 B written to the slab, read back once by the draws)
  + frame output (batch sums 28 B per unit written and read, the framebuffer 24 B per pixel) / rays
and traffic / algorithmic, the fraction of those bytes the caches did NOT serve.  build_id = rp_build_id() of the
library that ran the passes: bench.py refuses a record of another build.
"""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess

KERNEL = "render_kernel<false, "  # the frame kernel (either stack variant), not the probe
SIMDS = 1024
PEAK_CLOCK = 2.4e9


def read_pass(d, all_dispatches=False):
    """{counter: value} of the frame kernel's dispatch in one pass (rows of a dispatch summed), and its
    duration in ns.  all_dispatches: every frame-kernel dispatch of the pass summed (frames in flight), the mean
    duration, and their count."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if KERNEL not in row["Kernel_Name"]:
                continue
            did = row["Dispatch_Id"]
            per[did][row["Counter_Name"]] += float(row["Counter_Value"])
            dur[did] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    if not per:
        raise SystemExit(f"no {KERNEL} rows under {d}")
    if all_dispatches:
        tot = collections.defaultdict(float)
        for v in per.values():
            for k, x in v.items():
                tot[k] += x
        return dict(tot), sum(dur.values()) / len(dur), len(per)
    if len(per) != 1:
        raise SystemExit(f"{d}: {len(per)} frame-kernel dispatches (expected one: --steps 1 --warmup 0)")
    did = next(iter(per))
    return dict(per[did]), dur[did], 1


def lanes_per_ray(diag, region):
    r = diag["regions"][region]
    return r["wave_execs_per_kray"] * r["lane_util"] * 64.0 / 1000.0


def algorithmic(diag, node_bytes, bench):
    """Algorithmic bytes per ray of the render kernel (module docstring) from a diagnostic record."""
    cfg = bench["config"]
    W, H, spp = cfg["width"], cfg["height"], cfg["spp"]
    rays = float(cfg["rays_per_frame"])
    nbatch = -(-spp // cfg.get("samples_per_stream", 32))
    out_bytes = (W * H * nbatch * 28 * (2 if nbatch > 1 else 0) + W * H * 24) / rays
    parts = {
        "nodes": diag["visits_per_ray"] * node_bytes,
        "prims": diag["prim_tests_per_ray"] * 80.0,
        "hit_records": lanes_per_ray(diag, "surface") * 232.0,
        "texels": lanes_per_ray(diag, "texture") * 4.0,
        "keystream": lanes_per_ray(diag, "refill") * 128.0,
        "output": out_bytes,
    }
    return {"algorithmic_bytes_per_ray": sum(parts.values()),
            "algorithmic_breakdown": {k: round(v, 2) for k, v in parts.items()},
            "diag": {"visits_per_ray": diag["visits_per_ray"], "prim_tests_per_ray": diag["prim_tests_per_ray"],
                     "node_bytes": node_bytes, "spp": diag.get("spp"), "phase_share": diag.get("phase_share")}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--bench", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--diag", help="tools/diag.py record of the same build and frame")
    ap.add_argument("--node-bytes", type=int, default=0, help="bytes one node visit loads (0: C5 -> 64 (q8), else 112)")
    ap.add_argument("--all-dispatches", action="store_true",
                    help="sum every frame-kernel dispatch of each pass (a run of several frames, e.g. shards in flight); "
                         "per-ray figures use rays_per_frame x dispatches")
    ap.add_argument("passes", nargs="+")
    a = ap.parse_args()
    bench = json.loads(open(a.bench).read().strip().splitlines()[-1])
    rays = float(bench["config"]["rays_per_frame"])
    sizes = bench.get("roofline", {}).get("frames_per_launch") or [1]  # frames of each launch (bench.py)
    if isinstance(sizes, int):
        sizes = [sizes]
    c, durs, ndisp = {}, {}, set()
    for d in a.passes:
        vals, ns, nd = read_pass(d, a.all_dispatches)
        c.update(vals)
        durs[os.path.basename(d.rstrip("/"))] = ns
        ndisp.add(nd)
    if len(ndisp) != 1:
        raise SystemExit(f"passes saw different dispatch counts {sorted(ndisp)}")
    nd = ndisp.pop()
    if nd == len(sizes):
        rays *= sum(sizes)  # the timed launches' frames
    elif len(set(sizes)) == 1:
        rays *= sizes[0] * nd  # launches of one size (warm-up launches included with --all-dispatches)
    else:
        raise SystemExit(f"{nd} dispatches per pass, the bench made {len(sizes)} launches {sizes}")
    rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    build = bench.get("roofline", {}).get("build_id")
    rec = {"kernel": KERNEL, "config": a.config, "git": rev or None, "build_id": build, "rays": rays,
           "samples_per_stream": bench["config"].get("samples_per_stream", 32),
           "frames_per_launch": sizes, "counters": c,
           "kernel_ns_per_pass": durs, "bench_ms_per_step": bench.get("ms_per_step")}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch, write = 2.0 * c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0
        rec.update({"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                    "traffic_bytes_per_ray": (fetch + write) / rays,
                    "fetch_bytes_per_ray": fetch / rays, "write_bytes_per_ray": write / rays})
    for k, name in (("SQ_INSTS_VALU", "valu_per_ray"), ("SQ_INSTS_SALU", "salu_per_ray"),
                    ("SQ_INSTS_VMEM_RD", "vmem_rd_per_ray"), ("SQ_INSTS_VMEM_WR", "vmem_wr_per_ray"),
                    ("SQ_INSTS_LDS", "lds_per_ray"), ("SQ_INSTS_SMEM", "smem_per_ray"),
                    ("SQ_INSTS_BRANCH", "branch_per_ray")):
        if k in c:
            rec[name] = c[k] / rays
    if all(k in c for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
        w = c["SQ_WAVE_CYCLES"]
        rec["cycle_budget"] = {
            "wait_any": round(c["SQ_WAIT_ANY"] / w, 4), "wait_inst_any": round(c["SQ_WAIT_INST_ANY"] / w, 4),
            "active_inst_any": round(c["SQ_ACTIVE_INST_ANY"] / w, 4),
            "closure": round((c["SQ_WAIT_ANY"] + c["SQ_WAIT_INST_ANY"] + c["SQ_ACTIVE_INST_ANY"]) / w, 4),
            "waves": c.get("SQ_WAVES")}
    if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_VALU" in c and not a.all_dispatches:
        ns = next((v for k, v in durs.items() if v > 0), None)
        if ns:
            clk = c["GRBM_GUI_ACTIVE"] / 8.0 / (ns * 1e-9)
            rec["clock_ghz"] = round(clk / 1e9, 3)
            rec["valu_issue_frac_at_clock"] = round(c["SQ_INSTS_VALU"] / (SIMDS * clk * ns * 1e-9 / 2.0), 4)
            rec["valu_issue_frac_at_2p4ghz"] = round(c["SQ_INSTS_VALU"] / (SIMDS * PEAK_CLOCK * ns * 1e-9 / 2.0), 4)
    mix = {k[len("SQ_INSTS_VALU_"):].lower(): c[k] / c["SQ_INSTS_VALU"] for k in c
           if k.startswith("SQ_INSTS_VALU_") and "SQ_INSTS_VALU" in c}
    if mix:
        rec["valu_mix"] = {k: round(v, 4) for k, v in sorted(mix.items())}
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
        rec["valu_thread_cycles_per_active_quad"] = round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 3)
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        rec["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    if a.diag:
        rec.update(algorithmic(json.load(open(a.diag)), a.node_bytes or (64 if a.config == "C5" else 112), bench))
        if "traffic_bytes_per_ray" in rec:
            rec["traffic_over_algorithmic"] = round(rec["traffic_bytes_per_ray"] / rec["algorithmic_bytes_per_ray"], 4)
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "counters"}))


if __name__ == "__main__":
    main()

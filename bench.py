"""Benchmark: Mrays/s of the MI355X path tracer on BASELINE.json's headline configuration.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one frame of the config (1920x1080x256 spp bunny scene with full materials by default),
tile-sharded across the N ranks (the balanced tile plan, RP_SHARD_BALANCED: tiles dealt by a learned cost; strong
scaling: the frame is fixed), rendered by the persistent HIP kernel (librp.so) from scene data resident in HBM, followed
by librp's frame gather (rp_frame_gather): to_srgb_u8 -> B, G, R, A bytes, one RCCL all-gather of those 4 bytes per
pixel over xGMI (one collective per launch for all its frames, rp_frames_gather), and the device-side de-interleave into
frame order on every rank (the body of the reference's output.tga), counters summed over the ranks by RCCL as well.  torch.distributed (gloo) only bootstraps the RCCL
communicator and takes the barrier and max-time reduction.  The K frames are a frame sequence rendered in launches of
at most L = 32 (--frames-per-launch; rp_render_frames_device_ws, frames interleaved in cost order, a pixel's frames
consecutive: RP_FRAME_ORDER_PIXEL): the process renders
ONE sequence -- warm-up, timed, single-frame and side-leg launches take its next frames, frame f the config's frame of
seed + f * B * W * H (B sample batches per pixel), so no timed frame repeats a warm-up frame's seeds -- every frame
traced, shaded and gathered in full.  `value` is that frame-sequence throughput: no frame of a launch is available
before the launch ends (~L x 0.2 s on C3); the rate of lone frames (one per launch) is reported beside it
(single_frame).  RNG contract: on one GPU SURVEY.md 8c's one stream per pixel (samples_per_stream = spp), with the
32-sample streams of N > 1 runs timed beside it (streams_of_32); N > 1: 32-sample streams, the one-stream contract
beside it (contract_one_stream).  With N > 1 up to three launches are in flight on their own streams and
workspaces (--inflight; an 8-way C3 shard: 26.0 / 25.9 / 25.7 ms per frame with 1 / 2 / 3).
The timed region is K steps bracketed by a barrier + torch.cuda.synchronize() on both sides; the max over ranks is
used.

Rays = root scene.hit() calls (render.rs:105,133), counted on the device; value = all ranks' rays / time.
roofline: per ray of the render kernel, from the committed profile record of THIS build
(profiles/current.json -> tools/roofline.py output, refused when its build id differs from rp_build_id()), times this
launch's rays, over the launch's duration (HIP events on its stream):
  achieved / frac = memory-side bytes from the PMC counters (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
             MI355X_MICROARCH.md; Infinity-Cache hits are counted, so an upper bound of HBM traffic) against the 8 TB/s
             HBM peak -- the HBM roofline fraction; traffic = those bytes per launch (kernel_ms: its mean duration; a
             launch renders frames_per_launch frames);
  binding_frac = the fraction of its own roof of what binds the kernel: the larger of the VALU pipe's busy fraction
             (valu_busy: AMD's VALUBusy from SQ_ACTIVE_INST_VALU) and frac;
  l2_level = the kernel's ALGORITHMIC bytes (its node visits x node bytes + primitive tests x 80 B + the closest hit's
             records + texels + keystream, from the diagnostic build's counts) at this rate, against the guide's
             measured L2-shared gather rate (16.8-18.8 TB/s): these bytes are served by L2 and the Infinity Cache;
and, for reference, the rate the reference's own traversal would need (its event counts x SURVEY.md 8d bytes per
event).  cpu_baseline: the CPU oracle's -O3 restatement of the reference driver (main.rs:36-106: LIFO tile queue,
worker threads with their own StdRng) on a bounded sample of the same scene at 1, 4 (the reference's main.rs:27
default), 8 and 16 workers (16 = the box's CPU share per GPU; a GPU job on this pool sizes its worker pools to it),
rank 0, N = 1 only; the full host is a least-squares line through those four measured points, evaluated at the
host's physical core count (an extrapolation, labelled so).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd")]

METRIC = "Mrays/s at 1920×1080×256spp bunny scene; 1/2/4/8-GPU scaling + %HBM roofline"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
SIMDS = 1024                 # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9             # MI355X_MICROARCH.md max clock
# a wave64 v_fma_f32 occupies a SIMD-32 for 2 cycles (MI355X_MICROARCH.md "Wave scheduling"): the issue ceiling if every
# instruction were that fast.  Most are not: tools/valu_rates.hip measured ~4.1 SIMD cycles per wave64 instruction for
# f64 ops, compares, selects, min/max, conversions, permutes and the packed f32 ops, ~2.3 only for f32 FMA/ADD/MUL, integer
# add/sub/logic, right shifts and moves (profiles/r6/valu_rates_gfx950.json) -- so the VALU pipe's busy fraction is read
# from the hardware (SQ_ACTIVE_INST_VALU, AMD's VALUBusy), not priced from instruction counts.
VALU_ISSUE_PEAK = SIMDS * CLOCK_HZ / 2.0
CUS = SIMDS // 4


def valu_busy_per_ray(rec):
    """SQ_ACTIVE_INST_VALU per ray (quad-cycles summed over the SIMDs: AMD's VALUBusy = it / CUs / cycles) and the VALU
    lane utilisation (SQ_THREAD_CYCLES_VALU / (it x 64)), or None when the record lacks them."""
    c = rec.get("counters", {})
    if "SQ_ACTIVE_INST_VALU" not in c or not c["SQ_ACTIVE_INST_VALU"]:
        return None
    util = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]) if "SQ_THREAD_CYCLES_VALU" in c else None
    return c["SQ_ACTIVE_INST_VALU"] / rec["rays"], util
# SURVEY.md 8d algorithmic bytes per event of the REFERENCE traversal (reference tree, f64 layout)
BYTES = {"box_tests": 56, "tri_tests": 84, "sphere_tests": 32, "tri_hits": 120, "texels": 4}
# MI355X_MICROARCH.md "Indexed rows": rows shared by every workgroup, gathered from the XCD's L2: 16.8-18.8 TB/s
L2_GATHER_GBS = 18800.0
# FP64 vector peak: half the FP32 vector rate (157.3 TFLOP/s, MI355X_MICROARCH.md); the guide lists no FP64 figure
FP64_VALU_PEAK_TFLOPS = 157.3 / 2
# (workers, spp) of the CPU baseline runs, ~13 s each: 1 worker; main.rs:27 num_workers = 4; 8; 16 = the GPU box's CPU
# share (the line through all four is the full-host extrapolation)
CPU_RUNS = ((1, 2), (4, 8), (8, 16), (16, 32))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def reference_equivalent(config: str):
    """Bytes per ray the reference's own traversal would fetch (tests/golden/event_counts.json)."""
    ev = json.load(open(os.path.join(REPO, "tests", "golden", "event_counts.json")))
    per = ev["C3" if config == "C4" else config]["per_ray"]
    return sum(BYTES[k] * per[k] for k in BYTES)


def kernel_record(config: str, sps: int):
    """The committed per-ray record of the current frame kernel for this config and RNG contract (profiles/current.json
    -> a tools/roofline.py record over rocprofv3 --pmc passes; key "<config>" or "<config>@<samples_per_stream>", the
    record's own samples_per_stream must match): memory-side bytes per ray, VALU / SALU instructions per ray, cycle
    budget."""
    try:
        cur = json.load(open(os.path.join(REPO, "profiles", "current.json")))["roofline"]
    except (OSError, KeyError):
        return None
    for key in (config, f"{config}@{sps}"):
        if key in cur:
            rec = json.load(open(os.path.join(REPO, cur[key])))
            if rec.get("samples_per_stream", 32) == sps:
                rec["source"] = cur[key]
                return rec
    return None


class stdout_to_stderr:
    """Route fd 1 to stderr while RCCL initialises: it prints a version banner on stdout, and rank 0's stdout
    must be exactly the one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        ctypes.CDLL(None).fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)


def host_cpu():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        phys = len({(l.split(":")[1].strip()) for l in open("/proc/cpuinfo") if l.startswith("core id")}) or None
        sockets = len({(l.split(":")[1].strip()) for l in open("/proc/cpuinfo") if l.startswith("physical id")}) or 1
        phys = phys * sockets if phys else None
    except OSError:
        phys = None
    return {"model": model, "logical_cpus": os.cpu_count(), "physical_cores": phys,
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def fit_workers(runs):
    """Least-squares line rate = intercept + per_worker * workers through the measured CPU runs (not forced
    through 0), its R^2, and each run's rate per worker (how linear the scaling is)."""
    xs = [r["workers"] for r in runs]
    ys = [r["value"] for r in runs]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx
    a = my - b * mx
    ss_res = sum((y - (a + b * x)) ** 2 for x, y in zip(xs, ys))
    ss_tot = sum((y - my) ** 2 for y in ys)
    return {"intercept": round(a, 4), "per_worker": round(b, 4), "r2": round(1 - ss_res / ss_tot, 6) if ss_tot else 1.0,
            "points": n, "per_worker_at": {str(x): round(y / x, 4) for x, y in zip(xs, ys)}}


def cpu_baseline(config: str, runs_plan, spp_override: int = 0):
    """The reference driver restated (oracle, -O3, no per-event counters): 1920x1080 at each run's spp."""
    from oracle import oracle_py as O
    from rtpotato import scenes
    scene, params = scenes.config_scene(config)
    d = scene.desc()
    os_ = O.OracleScene(d.addr(), d, fast=True)
    cam = scene.camera.to_c()
    runs = []
    for workers, spp in runs_plan:
        spp = spp_override or spp
        secs, ctr, _ = os_.baseline(ctypes.addressof(cam), params.width, params.height, spp, params.max_bounce, 32,
                                    workers, params.seed)
        runs.append({"workers": workers, "spp": spp, "value": ctr["rays"] / secs / 1e6, "seconds": round(secs, 3),
                     "rays": ctr["rays"]})
        log(f"[rank 0] cpu baseline {workers} workers, {spp} spp: {runs[-1]['value']:.2f} Mrays/s in {secs:.1f}s")
    os_.close()
    host = host_cpu()
    main = max(runs, key=lambda r: r["workers"])
    out = {"value": main["value"], "unit": "Mrays/s", "cores": main["workers"], "kind": "port",
           "sample": f"{config} scene {params.width}x{params.height} at {', '.join(str(r['spp']) for r in runs)} spp for "
                     f"{', '.join(str(r['workers']) for r in runs)} workers (GPU runs {params.spp}spp); C restatement "
                     f"(-O3, oracle/liboracle_fast.so) of main.rs:36-106: LIFO tile queue of 32x32 tiles, one StdRng "
                     f"per worker (main.rs:27 default 4 workers); value = the {main['workers']}-worker run (the GPU "
                     f"box's CPU share); Rust reference unbuildable here",
           "runs": runs, "host": host}
    phys = host.get("physical_cores")
    if phys and len(runs) >= 3:
        fit = fit_workers(runs)
        out["full_host_extrapolated"] = {
            "value": round(fit["intercept"] + fit["per_worker"] * phys, 2), "cores": phys, "fit": fit,
            "basis": f"least-squares line through the {fit['points']} measured worker counts "
                     f"{[r['workers'] for r in runs]} evaluated at {phys} physical cores; not run -- a GPU job on this "
                     f"pool sizes its worker pools to its {main['workers']}-core share"}
    return out


def launch_sizes(n: int, per_launch: int, min_launches: int = 0) -> list:
    """n frames in the fewest launches of <= per_launch frames (at least min_launches), sizes as equal as they can be:
    20 frames, 8 per launch -> [7, 7, 6]."""
    parts = max(-(-n // per_launch), min_launches) if n > 0 else 0
    return [n // parts + (1 if j < n % parts else 0) for j in range(parts)]


# resident lanes of a launch, at most: 256 CUs x 32 one-wave blocks x 64 lanes (rp_api.cpp render_shard's queue bound)
LANES_MAX = 256 * 32 * 64


def frames_per_launch_cap(per_launch: int, slots: int, batches: int, lanes: int = LANES_MAX) -> int:
    """Frames per launch, at most what rp_api.cpp render_shard accepts for a launch of n = slots x sample batches x
    frames units: n < 2^31 (the unit decode) and, with per-XCD queues, 2 n + resident lanes < 2^32 - 1 (a queue word
    takes its units plus one failed fetch per lane and per drained queue passed): a C5 frame (16.8 M pixels of 8
    batches) takes at most 15 a launch."""
    units = min((1 << 31) - 1, (0xFFFFFFFE - lanes) // 2)
    return max(1, min(per_launch, units // (max(1, slots) * max(1, batches))))


U64 = (1 << 64) - 1


def frame_seed(seed: int, nbatch: int, width: int, height: int, f: int) -> int:
    """The RNG-contract seed of frame f of a frame sequence (rp_render_frames_device_ws: frame f of a launch whose
    params carry `seed` renders with seed + f * B * W * H, B = sample batches per pixel), wrapping like u64."""
    return (seed + f * nbatch * width * height) & U64


class FrameSeq:
    """The frame sequence of one process: every launch renders the next frames of it, so warm-up, timed, single-frame
    and side-leg frames have disjoint seeds -- the timed frames' tile costs are learned from earlier
    frames, as in a real sequence.  launch(p, n) -> the params whose launch renders frames f0 .. f0 + n - 1."""

    def __init__(self):
        self.next = 0

    def launch(self, seed: int, nbatch: int, width: int, height: int, n: int) -> tuple:
        f0 = self.next
        self.next += n
        return f0, frame_seed(seed, nbatch, width, height, f0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)  # one launch of 16 frames
    ap.add_argument("--warmup", type=int, default=8)  # spread over the in-flight workspaces: each learns its tile costs
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp (0 = config)")
    ap.add_argument("--samples-per-stream", type=int, default=0,
                    help="rp_render_params.samples_per_stream, the RNG contract (0 = auto: SURVEY.md 8c's one stream "
                         "per pixel, = spp, on one GPU; RP_SAMPLES_PER_STREAM = 32 for N > 1 and --shard-of; >= spp: "
                         "one stream per pixel)")
    ap.add_argument("--tile", type=int, default=0,
                    help="tile side in pixels (rp_render_params.tile_w/tile_h; 0 = the config's 32): scheduling only, "
                         "the image does not depend on it")
    ap.add_argument("--cpu-spp", type=int, default=0, help="override the CPU baseline runs' spp (0 = per run)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight: consecutive frames alternate over this many streams and workspaces "
                         "(0 = 1 on one GPU, 3 on several)")
    ap.add_argument("--frames-per-launch", type=int, default=32,
                    help="frames rendered by one persistent launch (rp_render_frames_device_ws: frame f of a launch is "
                         "the frame of seed + f * B * W * H); a step is still one frame (K frames in launches of <= L)")
    ap.add_argument("--frame-order", default="pixel", choices=("sequential", "interleaved", "pixel"),
                    help="RP_FRAME_ORDER_* of a launch of several frames (pixel: interleaved with a pixel's frames "
                         "consecutive, C3 -0.66 %% against interleaved, profiles/r6/c3_v58_knob_sweep_ab.json)")
    ap.add_argument("--no-single-frame", action="store_true",
                    help="skip the single-frame-per-launch timing reported beside a frame-sequence headline")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic, one GPU: render only shard --shard of this many (the per-rank work of an N-GPU "
                         "run), no gather; not a bench line")
    ap.add_argument("--shard", type=int, default=0, help="with --shard-of: which shard")
    ap.add_argument("--shard-map", default="auto", choices=("auto", "interleave", "balanced"),
                    help="tile deal across ranks (rp_render_params.shard_map); auto = balanced for N > 1 or --shard-of")
    ap.add_argument("--contract-steps", type=int, default=-1,
                    help="frames timed after the headline under the other RNG contract: 32-sample streams when the "
                         "headline is SURVEY.md 8c's one stream per pixel (N = 1), reported as streams_of_32, else the "
                         "one-stream contract, reported as contract_one_stream (-1 = a launch's worth for the default "
                         "workload, 0 = off)")
    ap.add_argument("--opt", action="append", default=[],
                    help="rp_scene_options field=value (tuning; e.g. --opt trav_threshold=20)")
    args = ap.parse_args()
    L = args.frames_per_launch
    if not 1 <= L <= 64 or args.steps < 1:
        ap.error("--frames-per-launch must be 1..64 (RP_MAX_FRAMES), --steps >= 1")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rank 0's stdout is the one JSON line: every other write to fd 1 (torch, gloo, RCCL, HIP -- on every rank) goes to
    # stderr for the whole run, and the line goes out through a private copy of the original stdout
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    # Rehearsal (tests/test_gpu_bench_rehearsal.py): RP_BENCH_REHEARSAL=gloo runs the N-rank loop with every rank on
    # device 0 and the frames gathered by rp_frames_pack -> a gloo all-gather of the packed blocks -> rp_frames_unpack
    # (RCCL puts no two ranks on one device).  It exercises this loop's N > 1 code on a one-GPU box; its line is labelled
    # and is not a measurement.
    rehearsal = world > 1 and os.environ.get("RP_BENCH_REHEARSAL", "") == "gloo"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        with stdout_to_stderr():  # gloo logs its peer connections on stdout
            dist.init_process_group("gloo")  # bootstrap + barrier + max-time only; frames move over librp's RCCL

    from dataclasses import replace
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import bootstrap_comm, shard_params
    from rtpotato.render import DeviceScene

    options = {}
    for kv in args.opt:
        k, v = kv.split("=", 1)
        options[k] = float(v) if k == "cost_traverse" else (v if k in ("builder", "node_format", "tile_order", "unit_queues", "collapse", "node_layout", "unit_order") else int(v))
    scene, params = scenes.config_scene(args.config)
    if args.spp:
        params = replace(params, spp=args.spp)
    # The RNG contract: on one GPU the headline is SURVEY.md 8c's contract itself -- one
    # StdRng::seed_from_u64(seed + j W + i) per pixel running main.rs:70-86 over all spp -- which renders C3 as fast as
    # 32-sample streams once a launch holds a frame sequence (BENCH_r05: 196.4 vs 198.4 ms).  N > 1 keeps 32-sample
    # streams: an 8-way shard of one-stream units is ~1 unit per resident lane and ran 9 % slower.
    sps_auto = args.samples_per_stream == 0 and world == 1 and not args.shard_of
    if args.samples_per_stream or sps_auto:
        params = replace(params, samples_per_stream=args.samples_per_stream or params.spp)
    if args.tile:
        params = replace(params, tile_w=args.tile, tile_h=args.tile)
    t = time.time()
    ds = DeviceScene(scene, device=local, options=options)
    info = ds.info()
    log(f"[rank {rank}] scene ready in {time.time() - t:.2f}s: {info}")
    nsh = args.shard_of or world
    smap = args.shard_map if args.shard_map != "auto" else ("balanced" if nsh > 1 else "interleave")
    params = replace(params, shard_map=F.RP_SHARD_BALANCED if smap == "balanced" else F.RP_SHARD_INTERLEAVE)
    sp = shard_params(params, rank, world) if not args.shard_of else shard_params(params, args.shard, args.shard_of)
    comm = None
    if not rehearsal:
        with stdout_to_stderr():
            comm = bootstrap_comm(rank, world, local)
    # Frames per launch (rp_render_frames_device_ws): one persistent launch renders L frames, frame f of
    # it the frame of seed + f * B * W * H, and hands out the frames' k-th tiles of the cost order together
    # (RP_FRAME_ORDER_INTERLEAVED).  The GPU's 262,144 resident lanes hold 1.6 % of a C3 frame's 16.6 M units and 12.5 %
    # of an 8-way shard's: the wider the band of the cost order in flight, the more lanes of a wave idle beside longer
    # paths (VALU / ray +10 %, L2 hit rate 0.72 vs 0.75 for a shard).  Interleaving L frames narrows the band L times:
    # C3 207.1 -> 202.5 ms per frame at L = 8, an 8-way shard 28.6 -> 26.1 ms, the one-stream contract 261 -> 204 ms
    # (profiles/r5/c3_frames_per_launch_ab.json); with one tile of every frame per queue chunk (v56) C3 205.3 / 199.4 /
    # 198.5 / 197.2 ms at L = 1 / 8 / 16 / 32 (c3_frames_chunk_auto_sweep.json, c3_frames_per_launch_large.json).  A step
    # is still one frame: K steps = K frames in the fewest launches of <= L.  The driver's 20 steps: one launch of 20 at
    # L = 32, 198.3 ms per frame, against two of 10 at L = 16, 199.1 ms; an 8-way shard's projected N = 8 efficiency
    # 0.976 vs 0.973 (profiles/r5/c3_v57_driver_cmd_L{16,32}_bench.json, c3_v57_scale_projection_pl{10,20}_f20.json).
    # Frames in flight: launch k renders on stream k % F with its own workspace and shard buffers; the frame gathers
    # (RCCL collectives) run on the main stream in frame order.  F = 1 is the plain sequential loop, whose launch
    # duration (HIP events, the rocprofv3 kernel trace) is the time of its L frames the roofline is priced on.
    from rtpotato.scene import shard_slot_count
    L = frames_per_launch_cap(L, shard_slot_count(sp),
                              -(-params.spp // (params.samples_per_stream or F.RP_SAMPLES_PER_STREAM)))
    F_ = args.inflight if args.inflight > 0 else (1 if world == 1 else 3)
    order = args.frame_order
    main_stream = torch.cuda.current_stream(dev)
    streams = [main_stream] if F_ == 1 else [torch.cuda.Stream(dev) for _ in range(F_)]
    wss = [None] + [ds.workspace() for _ in range(F_ - 1)]
    for w in wss:
        ds.reserve_frames(sp, L, w)  # batch sums + gather staging: nothing is allocated inside the timed loop
    from rtpotato.scene import shard_slot_count
    nslots = shard_slot_count(sp)
    n3 = 3 * max(1, nslots)
    bufs = [torch.zeros(n3 * L, dtype=torch.float64, device=dev) for _ in range(F_)]
    ctrs = [torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev) for _ in range(F_)]
    nfr = [1] * F_  # frames of the buffer's last launch (its counters are their sums)
    freed = [None] * F_  # event: the gathers of the buffer's previous launch are done
    frames = torch.zeros(params.height * params.width * 4 * L, dtype=torch.uint8, device=dev)  # a launch's frames
    state = {"k": 0}
    launches_all = []  # (frames, start, end) of every launch of this process, warm-up and side runs included
    seq = FrameSeq()  # warm-up, timed, single-frame and side-leg frames: one sequence, disjoint seeds

    def step(n, k_start=None, k_end=None, spx=None):
        """One launch of n <= L frames (the next n of the process's frame sequence) on the next workspace, then their
        gathers."""
        spx = spx if spx is not None else sp
        nb = -(-spx.spp // (spx.samples_per_stream or F.RP_SAMPLES_PER_STREAM))
        spx = replace(spx, seed=seq.launch(spx.seed, nb, spx.width, spx.height, n)[1])
        i = state["k"] % F_
        state["k"] += 1
        st = streams[i]
        if freed[i] is not None:
            st.wait_event(freed[i])
        if k_start is None:
            k_start, k_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        launches_all.append((n, k_start, k_end))
        k_start.record(st)
        if L == 1:
            ds.render_device(spx, bufs[i], ctrs[i], stream=st, workspace=wss[i])
        else:
            ds.render_frames_device(spx, n, bufs[i], ctrs[i], stream=st, workspace=wss[i], order=order)
        nfr[i] = n
        k_end.record(st)
        if st is not main_stream:
            done = torch.cuda.Event()
            done.record(st)
            main_stream.wait_event(done)
        if args.shard_of:
            freed[i] = done if st is not main_stream else None
            return
        # the launch's frames: output stage + ONE RCCL all-gather of their BGRA8 shards + de-interleave into n frames
        # (+ the launch's counters summed over the ranks), on the main stream
        if rehearsal:
            send = torch.zeros(ds.frames_block_words(spx, n), dtype=torch.int32, device=dev)
            ds.frames_pack(spx, n, bufs[i], ctrs[i], send, stream=main_stream, workspace=wss[i])
            main_stream.synchronize()
            blocks = [torch.zeros(send.numel(), dtype=torch.int32) for _ in range(world)]
            dist.all_gather(blocks, send.cpu())
            recv = torch.cat(blocks).to(dev)
            ds.frames_unpack(spx, n, recv, frames, counters=ctrs[i], stream=main_stream, workspace=wss[i])
        elif L == 1:
            ds.frame_gather(comm, spx, bufs[i], frame_bgra=frames, counters=ctrs[i], stream=main_stream,
                            workspace=wss[i])
        else:
            ds.frames_gather(comm, spx, n, bufs[i], frames_bgra=frames, counters=ctrs[i], stream=main_stream,
                             workspace=wss[i])
        freed[i] = torch.cuda.Event()
        freed[i].record(main_stream)

    def run(spx, nframes, events=True, per_launch=None):
        """nframes frames in launches of <= per_launch (default L) frames (max-over-ranks seconds, launch events, rays
        per frame, samples)."""
        sizes = launch_sizes(nframes, per_launch or L)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in sizes]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for n, (s0, s1) in zip(sizes, ev):
            step(n, s0 if events else None, s1 if events else None, spx=spx)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tm = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        cs = [c.cpu().tolist() for c in ctrs]
        bad = [c[3] for c in cs if c[3] != 0]
        if bad:  # RP_STATUS_* bits (OR-ed over the ranks by the gather): stack overflow, plan mismatch
            raise RuntimeError(f"render kernel reported status {bad}: frame refused")
        last = (state["k"] - 1) % F_  # summed over the ranks by rp_frame_gather
        return (float(tm.item()), [s0.elapsed_time(s1) / 1e3 for s0, s1 in ev] if events else None,
                cs[last][0] / nfr[last], cs[last][1] / nfr[last], sizes)

    # warm-up: W frames over min(F, W) launches at least -- every in-flight workspace learns its tile costs
    for w, n in enumerate(launch_sizes(args.warmup, L, min(F_, args.warmup))):
        step(n)
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup launch {w} ({n} frames) done")
    elapsed_max, kdur, rays_step, samples_step, sizes = run(sp, args.steps)
    dump = os.environ.get("RP_BENCH_DUMP")
    if dump and rank == 0 and not args.shard_of:  # tests only: the timed run's last launch, assembled BGRA8 frames
        import numpy as np
        np.save(dump, frames[:sizes[-1] * params.width * params.height * 4].cpu().numpy())
    kernel_s = sum(kdur) / args.steps  # per frame: launch durations over the frames they rendered
    kernel_launch_ms = sum(kdur) / len(kdur) * 1e3
    if F_ > 1:
        # overlapping launches: a launch's events also span the neighbours' work, so the kernel rate is priced on the
        # per-frame throughput time instead
        kernel_s = elapsed_max / args.steps
    value = rays_step * args.steps / elapsed_max / 1e6

    # single-frame latency beside the frame-sequence throughput: one frame per launch, sequential, same workspaces
    single = None
    if L > 1 and not args.no_single_frame:
        nsf = 3
        for _ in range(F_):  # one lone frame per workspace first: it learns the unit durations a lone frame schedules
            step(1)          # by (rp_scene_options.unit_order AUTO: one stream per pixel)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(nsf):
            step(1)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tm = torch.tensor([time.perf_counter() - t1], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        r1 = ctrs[(state["k"] - 1) % F_][0].item()
        single = {"frames": nsf, "ms_per_frame": round(float(tm.item()) / nsf * 1e3, 3),
                  "value": round(r1 * nsf / float(tm.item()) / 1e6, 3), "unit": "Mrays/s",
                  "note": "one frame per launch (rp_render_frames_device_ws, n_frames 1) on the same streams and "
                          "workspaces, after one untimed lone frame per workspace: the rate of lone frames (the learned "
                          "unit order under one stream per pixel); the headline renders frame sequences of "
                          "frames_per_launch frames per launch"}

    # The other RNG contract, timed the same way after the headline frames: with the one-stream headline (N = 1) the
    # 32-sample streams N > 1 runs use (streams_of_32), else SURVEY.md 8c's contract itself (contract_one_stream: one
    # StdRng stream per pixel running the unchanged body of main.rs:70-86 over all spp).
    side, side_key = None, None
    one_stream = params.samples_per_stream >= params.spp
    side_sps = F.RP_SAMPLES_PER_STREAM if one_stream else params.spp
    # the side contract's own launch cap: 32-sample streams carry spp / 32 units per pixel (C5: 15 frames a launch)
    Lc = frames_per_launch_cap(L, nslots, -(-params.spp // side_sps))
    csteps = args.contract_steps if args.contract_steps >= 0 else (
        (Lc if Lc > 1 else 3) if (sps_auto or not args.samples_per_stream) and not (args.shard_of or args.spp or args.tile)
        else 0)
    if csteps > 0 and params.spp > F.RP_SAMPLES_PER_STREAM:
        side_key = "streams_of_32" if one_stream else "contract_one_stream"
        spc = shard_params(replace(params, samples_per_stream=side_sps), rank, world)
        for w in wss:
            ds.reserve_frames(spc, Lc, w)
        for _ in range(F_):  # one launch per in-flight workspace: each learns this contract's tile costs
            step(1, spx=spc)
            torch.cuda.synchronize()
        tcs, _, crays, _, csz = run(spc, csteps, events=False, per_launch=Lc)
        side = {"samples_per_stream": side_sps, "steps": csteps, "warmup": F_, "launches": csz,
                "ms_per_step": round(tcs / csteps * 1e3, 3),
                "value": round(crays * csteps / tcs / 1e6, 3), "unit": "Mrays/s",
                "rays_per_frame": int(crays),
                "note": ("the 32-sample streams (RP_SAMPLES_PER_STREAM) that N > 1 runs use: batch b of a pixel is "
                         "StdRng::seed_from_u64(seed + b*W*H + j*W + i); the headline is SURVEY.md 8c's one stream per "
                         "pixel") if one_stream else
                        ("SURVEY.md 8c: one StdRng::seed_from_u64(seed + j*W + i) stream per pixel over all spp "
                         "(main.rs:70-86 unchanged); the headline uses streams of samples_per_stream samples")}

    if rank == 0:
        local_rays = rays_step / world  # this rank's launch (shards carry near-equal work under the balanced plan)
        # the per-ray record is of the default workload (its spp, RNG contract and tile size)
        rec = kernel_record(args.config, params.samples_per_stream or F.RP_SAMPLES_PER_STREAM) \
            if args.spp == 0 and args.tile == 0 else None
        build = F.rp().rp_build_id().decode()
        roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None,
                "kernel": "rpk::render_kernel<false, *>", "kernel_ms": round(kernel_launch_ms, 3),
                # every launch of this process (warm-up, timed, single_frame, contract): what a rocprofv3 kernel summary of
                # the same command averages
                "kernel_ms_all_launches": round(sum(a.elapsed_time(b) for _, a, b in launches_all) / len(launches_all), 3),
                "launches_all": [nn for nn, _, _ in launches_all],
                "kernel_ms_per_frame": round(kernel_s * 1e3, 3), "frames_per_launch": sizes, "build_id": build}
        fpl = args.steps / len(sizes)  # frames per launch, mean
        if rec and rec.get("build_id") != build:
            roof["stale_record"] = f"{rec['source']} was measured on build {rec.get('build_id')}; not used"
            rec = None
        binding = None
        if rec:
            traffic = rec["traffic_bytes_per_ray"] * local_rays * fpl  # per launch
            tr_gbs = traffic / fpl / kernel_s / 1e9
            tr_frac = tr_gbs / HBM_PEAK_GBS
            issue = rec["valu_per_ray"] * local_rays / kernel_s
            valu_frac = issue / VALU_ISSUE_PEAK
            roof.update({
                "achieved": round(tr_gbs, 1), "frac": round(tr_frac, 4), "traffic": round(traffic),
                "basis": "memory-side bytes of the launch (PMC: 2 x FETCH_SIZE + WRITE_SIZE per ray x this launch's "
                         "rays) / its HIP-event duration; Infinity-Cache hits included (an upper bound of HBM bytes)",
                "traffic_bytes_per_ray": round(rec["traffic_bytes_per_ray"], 1),
                "fetch_bytes_per_ray": round(rec["fetch_bytes_per_ray"], 1) if "fetch_bytes_per_ray" in rec else None,
                "write_bytes_per_ray": round(rec["write_bytes_per_ray"], 1) if "write_bytes_per_ray" in rec else None,
                "valu_issue": {"achieved": round(issue / 1e9, 1), "peak": round(VALU_ISSUE_PEAK / 1e9, 1),
                               "unit": "Gwave-inst/s", "frac": round(valu_frac, 4),
                               "valu_per_ray": round(rec["valu_per_ray"], 2)},
                "cycle_budget": rec.get("cycle_budget"),
                "source": f"{rec['source']} (rocprofv3 PMC + diagnostic counts, build {rec.get('build_id')}; per-ray "
                          f"figures x this launch's rays / its HIP-event duration)"})
            alg = rec.get("algorithmic_bytes_per_ray")
            if alg:
                l2 = alg * local_rays / kernel_s / 1e9
                roof["l2_level"] = {
                    "achieved": round(l2, 1), "peak": L2_GATHER_GBS, "unit": "GB/s", "frac": round(l2 / L2_GATHER_GBS, 4),
                    "bytes_per_ray": round(alg, 1), "breakdown": rec.get("algorithmic_breakdown"),
                    "traffic_over_algorithmic": round(rec["traffic_bytes_per_ray"] / alg, 4),
                    "note": "the kernel's own algorithmic bytes (what its loads touch), served by L2 / Infinity Cache; "
                            "peak = MI355X_MICROARCH.md's L2-shared row gather, 16.8-18.8 TB/s (upper end used)"}
            c = rec.get("counters", {})
            if all(k in c for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")):
                # % FP64-VALU roofline beside % HBM -- wave-instructions x 64 lanes, i.e. an upper bound
                # (inactive lanes counted), per ray of the record x this launch's rays
                f64_per_ray = 64.0 * (2.0 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                                      c["SQ_INSTS_VALU_ADD_F64"] + c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)) / rec["rays"]
                tf = f64_per_ray * local_rays / kernel_s / 1e12
                roof["fp64_valu"] = {"achieved": round(tf, 2), "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                                     "frac": round(tf / FP64_VALU_PEAK_TFLOPS, 4),
                                     "note": "upper bound: f64 FMA (2 flops), MUL, ADD, transcendental wave-instructions "
                                             "x 64 lanes; peak = half the FP32 vector rate (spec)"}
            vb = valu_busy_per_ray(rec)
            busy = None
            if vb is not None:
                busy = vb[0] * local_rays / kernel_s / (CUS * CLOCK_HZ)
                roof["valu_busy"] = {
                    "frac": round(busy, 4), "lane_utilisation": round(vb[1], 4) if vb[1] is not None else None,
                    "active_quad_cycles_per_ray": round(vb[0], 2),
                    "basis": "AMD's VALUBusy: SQ_ACTIVE_INST_VALU (quad-cycles, summed over the SIMDs) per ray of the record "
                             "x this launch's rays / (CUs x clock x launch duration); lane_utilisation = "
                             "SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64).  It counts one quad-cycle per VALU "
                             "instruction (calibrated: profiles/r6/valu_rates_gfx950.json), and full-rate ops may pair two "
                             "per quad-cycle (C3: SQ_ACTIVE_INST_VALU2 0.08), so it reads VALU issue, not pipe saturation",
                    "sensitivity": "16 extra VALU instructions per node visit cost 0.45 of their pipe time (v_fma_f32 "
                                   "+0.96 %, v_max_f32 +1.88 %; profiles/r6/c3_v58_valu_sensitivity_ab.json): VALU work "
                                   "the kernel sheds pays back about half its issue time"}
            vbind = busy if busy is not None else valu_frac
            binding = (("valu_busy" if busy is not None else "valu_issue"), vbind) if vbind >= tr_frac \
                else ("hbm_traffic", tr_frac)
            roof["binding"] = {"resource": binding[0], "frac": round(binding[1], 4),
                               "unweighted_valu_issue": round(valu_frac, 4),
                               "note": "VALU instructions issue in ~0.8-0.9 of the quad-cycles at ~0.47 lane utilisation (idle lanes of divergent "
                                       "traversal and shading); memory-side traffic is ~0.2 of HBM"}
        ref_bpr = reference_equivalent(args.config)
        roof["reference_equivalent"] = {
            "bytes_per_ray": round(ref_bpr, 1), "GBps": round(ref_bpr * local_rays / kernel_s / 1e9, 1),
            "note": "bytes the reference's own traversal (its median-split tree, 1 primitive per leaf, f64 "
                    "boxes) would fetch per ray at this ray rate; not traffic and not a roofline fraction"}
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "note": "frame-sequence throughput: the K timed frames in launches of frames_per_launch (no frame is "
                    "available before its launch ends); single_frame = one frame per launch (lone-frame latency)",
            "data": "reference assets (bunny.obj, earthmap.tga packed in-repo) + synthesized sky panorama",
            "config": {"workload": f"{args.config}: {scenes.CONFIGS[args.config].description}",
                       "width": params.width, "height": params.height, "spp": params.spp,
                       "max_bounce": params.max_bounce, "seed": params.seed,
                       "samples_per_stream": params.samples_per_stream or 32,
                       "rng_contract": "SURVEY.md 8c: one stream per pixel" if one_stream else
                                       f"streams of {params.samples_per_stream or 32} samples",
                       "tile": [params.tile_w, params.tile_h],
                       "parallelism": (f"REHEARSAL: {world} ranks on device 0, rp_frames_pack blocks all-gathered over "
                                       f"gloo (RP_BENCH_REHEARSAL; not a measurement)") if rehearsal else
                                      f"tile-sharded x{world} + RCCL all-gather (librp)" if world > 1 else "1 GPU",
                       "frames_in_flight": F_, "frames_per_launch": L,
                       "output": "to_srgb_u8 BGRA8 frame (TGA pixel order) assembled on every rank",
                       "rays_per_frame": int(rays_step), "rays_per_sample": rays_step / samples_step,
                       "msamples_per_s": round(samples_step * args.steps / elapsed_max / 1e6, 1),
                       "scene_options": options or "defaults", "shard_map": smap,
                       **({"simulated_shard": f"shard {args.shard} of {args.shard_of}, no gather (diagnostic)"}
                          if args.shard_of else {})},
            **({"rehearsal": True} if rehearsal else {}),
            "roofline": roof,
            "binding_frac": round(binding[1], 4) if binding else None,
            "binding_resource": binding[0] if binding else None,
            "cpu_baseline": None,
            "single_frame": single,
            **({side_key: side} if side_key else {}),
        }
        if world == 1 and not args.no_cpu_baseline and not args.shard_of:
            log("[rank 0] cpu baseline ...")
            cb = cpu_baseline(args.config, CPU_RUNS, args.cpu_spp)
            out["cpu_baseline"] = cb
            ratios = {f"vs_{r['workers']}_workers": round(value / r["value"], 1) for r in cb["runs"]}
            if "full_host_extrapolated" in cb:
                ratios["vs_full_host_extrapolated"] = round(value / cb["full_host_extrapolated"]["value"], 1)
            out["gpu_over_cpu"] = ratios
        line_out.write(json.dumps(out) + "\n")
        line_out.flush()
    if comm is not None:
        comm.close()
    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

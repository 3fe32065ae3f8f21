"""One-GPU number for the RCCL-LDS hazard: how long a collective's kernel waits for a CU
while frames are in flight.

bench.py's N > 1 loop renders frame k on stream k % 3 and runs frame k's gather (RCCL all-gather kernels) on the main
stream once frame k's render is done, while frames k + 1 and k + 2 render.  A persistent render block holds ~10 KB of
LDS and its wave 120 VGPRs until its last unit ends, 16 blocks per CU; RCCL's all-gather kernel on gfx950
(ncclDevKernel_Generic, librccl.so.1's gfx950 code object) needs 37,664 B of LDS per block and 256 VGPRs per lane, so
it can only start on a CU that several render waves have left.  With one GPU there is no RCCL all-gather kernel (a
1-rank communicator copies), so this tool enqueues, in place of the gather, a kernel of that footprint
(tools/lds_probe.hip: `--blocks` blocks of `--threads` threads, `--lds` bytes) behind a stamp kernel on the main stream,
and reads each block's start on the 100 MHz real-time clock: wait = block start - the moment the stream reached it.

    python tools/gather_lds_wait.py --config C3 --shard-of 8 --shard 3 --inflight 3 --frames 12 --blocks 32
"""
import argparse
import ctypes
import json
import os
import sys
import time
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracing-potato_amd"), os.path.join(REPO, "tools")]


def run(ds, sp, F, frames, probe, blocks, threads, lds, table):
    import torch
    from rtpotato.scene import shard_slot_count
    dev = torch.device("cuda", 0)
    main = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    wss = [ds.workspace() for _ in range(F)]
    for w in wss:
        ds.reserve(sp, w)
        if table is not None:
            ds.set_tile_costs(sp, table, sp.num_shards, w)
    n = shard_slot_count(sp)
    bufs = [torch.zeros(3 * max(1, n), dtype=torch.float64, device=dev) for _ in range(F)]
    ctrs = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(F)]
    outs = torch.zeros((frames, 1 + blocks), dtype=torch.int64, device=dev)
    freed = [None] * F
    lib = ctypes.CDLL(os.path.join(REPO, "raytracing-potato_amd", "lib", "liblds_probe.so"))
    lib.lds_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

    def frame(k, record):
        i = k % F
        st = streams[i]
        if freed[i] is not None:
            st.wait_event(freed[i])
        ds.render_device(sp, bufs[i], ctrs[i], stream=st, workspace=wss[i])
        done = torch.cuda.Event()
        done.record(st)
        main.wait_event(done)
        if probe and record:
            assert lib.lds_probe_launch(outs[k].data_ptr(), blocks, threads, lds, ctypes.c_void_p(main.cuda_stream)) == 0
        freed[i] = torch.cuda.Event()
        freed[i].record(main)

    for k in range(F):  # warm-up round: every workspace learns its costs
        frame(k, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(frames):
        frame(k, True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / frames
    assert all(int(c[3]) == 0 for c in ctrs)
    for w in wss:
        w.close()
    res = {"frame_ms": round(dt * 1e3, 3)}
    if probe:
        o = outs.cpu().numpy()
        first = (o[:, 1:].min(axis=1) - o[:, 0]) / 1e5
        last = (o[:, 1:].max(axis=1) - o[:, 0]) / 1e5
        res.update({"wait_first_block_ms": [round(float(x), 3) for x in first],
                    "wait_last_block_ms": [round(float(x), 3) for x in last],
                    "mean_wait_first_ms": round(float(first.mean()), 3),
                    "mean_wait_last_ms": round(float(last.mean()), 3), "max_wait_last_ms": round(float(last.max()), 3)})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--shard-of", type=int, default=8)
    ap.add_argument("--shard", type=int, default=3)
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--blocks", default="8,32", help="probe grid sizes (RCCL channels)")
    ap.add_argument("--threads", type=int, default=256)
    ap.add_argument("--lds", type=int, default=37664)
    ap.add_argument("--opt", action="append", default=[], help="rp_scene_options field=value")
    a = ap.parse_args()
    import torch  # noqa: F401
    from rtpotato import scenes
    from rtpotato.render import DeviceScene
    from shard_scaling import learned_table
    options = {k: int(v) for k, v in (kv.split("=", 1) for kv in a.opt)}
    scene, params = scenes.config_scene(a.config)
    ds = DeviceScene(scene, options=options)
    ds.render(replace(params, spp=4))
    params = replace(params, shard_map=1)
    table = learned_table(ds, params, a.shard_of) if a.shard_of > 1 else None
    sp = replace(params, shard=a.shard, num_shards=a.shard_of)
    out = {"config": a.config, "shard": f"{a.shard} of {a.shard_of} (balanced, learned table)", "inflight": a.inflight,
           "frames": a.frames, "probe": {"threads": a.threads, "lds_bytes": a.lds, "vgprs": 256,
                                         "source": "ncclDevKernel_Generic_{1,2,4} in librccl.so.1 (gfx950 code object)"},
           "scene_options": options or "defaults", "runs": {}}
    out["runs"]["no_probe"] = run(ds, sp, a.inflight, a.frames, False, 1, a.threads, a.lds, table)
    for b in [int(x) for x in a.blocks.split(",")]:
        out["runs"][f"probe_{b}_blocks"] = run(ds, sp, a.inflight, a.frames, True, b, a.threads, a.lds, table)
    out["runs"]["no_probe_again"] = run(ds, sp, a.inflight, a.frames, False, 1, a.threads, a.lds, table)
    ds.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

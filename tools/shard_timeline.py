"""Overlap of frames in flight in a kernel trace of tools/shard_scaling.py (gpu_session.sh step shardtrace_<CFG>):
per render launch its start, end and duration, and over the timed frames of each shard the time the GPU ran at least
one render, two or more at once, and none (gaps), plus what the other kernels between renders cost.

    python tools/shard_timeline.py gpurun_out/<tag>_<CFG>_shardtrace [--frames 6 --inflight 3]
"""
import argparse
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--inflight", type=int, default=3)
    a = ap.parse_args()
    f = glob.glob(f"{a.trace_dir}/**/*kernel_trace.csv", recursive=True)[0]
    ks = []
    for r in csv.DictReader(open(f)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])))
    ks.sort()
    renders = [k for k in ks if "render_kernel<false" in k[2]]
    # shard_scaling renders per shard: F warm-up frames then `frames` timed frames (the learned-table renders of the
    # first pass come before); take the timed group as the last `frames` of every F + frames block
    per = a.inflight + a.frames
    groups = []
    tail = renders[-8 * per:] if len(renders) >= 8 * per else renders
    for s in range(len(tail) // per):
        g = tail[s * per:(s + 1) * per][a.inflight:]
        groups.append(g)
    out = {"trace": f, "render_launches": len(renders), "shards": []}
    for g in groups:
        t0, t1 = g[0][0], max(k[1] for k in g)
        # coverage by renders
        ev = sorted([(k[0], 1) for k in g] + [(k[1], -1) for k in g])
        cur, last, one, two, none = 0, t0, 0, 0, 0
        for t, d in ev:
            span = t - last
            if cur == 0:
                none += span
            elif cur == 1:
                one += span
            else:
                two += span
            cur += d
            last = t
        others = [k for k in ks if t0 <= k[0] <= t1 and "render_kernel<false" not in k[2]]
        names = {}
        for k in others:
            n = k[2].split("(")[0][-40:]
            names.setdefault(n, [0, 0.0])
            names[n][0] += 1
            names[n][1] += (k[1] - k[0]) / 1e6
        span = (t1 - t0) / 1e6
        out["shards"].append({
            "span_ms": round(span, 3), "per_frame_ms": round(span / len(g), 3),
            "render_ms": [round((k[1] - k[0]) / 1e6, 2) for k in g],
            "one_render_ms": round(one / 1e6, 2), "two_plus_ms": round(two / 1e6, 2), "no_render_ms": round(none / 1e6, 2),
            "other_kernels": {n: {"n": v[0], "ms": round(v[1], 3)} for n, v in names.items()}})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

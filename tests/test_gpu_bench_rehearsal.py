"""bench.py's N > 1 loop, rehearsed on the one-GPU box (the loop had never executed).

The driver launches `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N` on an 8-GPU node.  RCCL
puts no two ranks on one device, so here every rank renders its tile shard on device 0 and the launch's frames are
gathered by the caller-collective pair of the C-ABI -- rp_frames_pack, a gloo all-gather of the packed blocks,
rp_frames_unpack (RP_BENCH_REHEARSAL=gloo) -- instead of librp's RCCL all-gather.  Everything else is the N-rank loop
itself: the gloo bootstrap, balanced shards, three launches in flight on their own streams and workspaces, the barriers
and the max-over-ranks time, the summed counters, rank 0's single JSON line -- and the frames it assembles, which must
equal the one-GPU run's bit for bit (per-unit seeding; RP_BENCH_DUMP saves the timed run's last launch).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


ARGS = ["--steps", "4", "--warmup", "2", "--spp", "40", "--samples-per-stream", "32", "--no-cpu-baseline"]


@pytest.fixture(scope="module")
def one_gpu_frames(tmp_path_factory):
    """The same command on one GPU (no rehearsal): its timed run's last launch, assembled."""
    out = str(tmp_path_factory.mktemp("n1") / "frames.npy")
    r = subprocess.run([sys.executable, "bench.py", *ARGS], cwd=REPO, env=dict(os.environ, RP_BENCH_DUMP=out),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    return np.load(out)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_rehearsal(gpu, world, one_gpu_frames, tmp_path):
    dump = str(tmp_path / "frames.npy")
    env = dict(os.environ, RP_BENCH_REHEARSAL="gloo", RP_BENCH_DUMP=dump)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(world), *ARGS]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]  # rank 0 alone prints: one JSON line
    d = json.loads(lines[0])
    assert d["rehearsal"] is True and "REHEARSAL" in d["config"]["parallelism"]
    assert d["n_gpus"] == world and d["steps"] == 4 and d["value"] > 0 and d["scaling"] == "strong"
    assert d["config"]["samples_per_stream"] == 32 and d["config"]["frames_in_flight"] == 3
    assert d["config"]["shard_map"] == "balanced"
    # the counters the unpack sums over the ranks: every pixel of the 1920 x 1080 frame once per sample
    assert d["config"]["rays_per_frame"] >= 1920 * 1080 * 40
    assert d["single_frame"] and d["single_frame"]["ms_per_frame"] > 0
    # the N-rank frames (balanced shards of 3 launches in flight, packed, gathered, assembled) = the one-GPU frames
    frames = np.load(dump)
    assert frames.shape == one_gpu_frames.shape and frames.size >= 1920 * 1080 * 4
    assert np.array_equal(frames, one_gpu_frames)

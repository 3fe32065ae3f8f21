"""Multi-process frames through the HIP path (the gloo tests in test_dist.py render with the
oracle).  Two processes share the one GPU of the box, one rank each, as bench.py's ranks would on two GPUs: every rank
builds its own device scene, renders its shard of the balanced tile plan with librp (the plan made independently on
each rank from the deterministic whole-frame probe), converts it to to_srgb_u8 bytes on the device
(rp_shard_to_bgra8), and the shards are all-gathered over gloo (RCCL cannot put two ranks on one device).  Rank 0
assembles the gathered shards on the device with its workspace's plan (rp_frame_assemble_ws), f64 and BGRA8 -- both
must equal the one-process rp_render frame bit for bit, and the ranks' plans must agree."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _params():
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    return RenderParams(150, 90, 6, 8, scenes.DEFAULT_SEED, 16, 16, shard_map=F.RP_SHARD_BALANCED)


def _worker(rank, world, port, result_dir):
    import ctypes
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "raytracing-potato_amd")]
    import torch
    import torch.distributed as dist
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import max_slots, shard_params
    from rtpotato.render import DeviceScene
    from rtpotato.scene import shard_slot_count
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    params = _params()
    scene = scenes.configure(scenes.bunny_full(), params.width, params.height)
    sp = shard_params(params, rank, world)
    S = max_slots(params, world)
    n = shard_slot_count(sp)
    with DeviceScene(scene, device=0) as ds:
        ws = ds.workspace()
        ds.reserve(sp, ws)
        rgb = torch.zeros(3 * S, dtype=torch.float64, device="cuda")
        bgra = torch.zeros(S, dtype=torch.int32, device="cuda")
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        ds.render_device(sp, rgb, ctr, workspace=ws)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        pc = sp.to_c()
        F.check(F.rp().rp_shard_to_bgra8(ds.handle, ctypes.byref(pc), rgb.data_ptr(), bgra.data_ptr(), st))
        torch.cuda.synchronize()
        assert int(ctr[3]) == 0 and n <= S
        plan = torch.as_tensor(ds.tile_map(sp, ws).astype(np.int64))
        plans = [torch.zeros_like(plan) for _ in range(world)]
        dist.all_gather(plans, plan)
        parts = [torch.zeros(3 * S, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, rgb.cpu())
        bparts = [torch.zeros(S, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(bparts, bgra.cpu())
        rays = ctr[:1].cpu()
        dist.all_reduce(rays)
        if rank == 0:
            g = torch.cat(parts).cuda()
            gb = torch.cat(bparts).cuda()
            frame = torch.zeros(params.width * params.height * 3, dtype=torch.float64, device="cuda")
            frame8 = torch.zeros(params.width * params.height, dtype=torch.int32, device="cuda")
            p0 = shard_params(params, 0, world).to_c()
            F.check(F.rp().rp_frame_assemble_ws(ds.handle, ws.handle, ctypes.byref(p0), g.data_ptr(), 6,
                                                frame.data_ptr(), st))
            F.check(F.rp().rp_frame_assemble_ws(ds.handle, ws.handle, ctypes.byref(p0), gb.data_ptr(), 1,
                                                frame8.data_ptr(), st))
            torch.cuda.synchronize()
            np.save(os.path.join(result_dir, "frame.npy"), frame.cpu().numpy().reshape(params.height, params.width, 3))
            np.save(os.path.join(result_dir, "frame8.npy"), frame8.cpu().numpy().view(np.uint8))
            np.save(os.path.join(result_dir, "plans.npy"), torch.stack(plans).numpy())
            np.save(os.path.join(result_dir, "rays.npy"), rays.numpy())
        ws.close()
    dist.destroy_process_group()


def test_two_process_hip_shards_rebuild_frame(gpu, tmp_path):
    from dataclasses import replace
    from rtpotato import _ffi as F
    from rtpotato import scenes
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    params = _params()
    scene = scenes.configure(scenes.bunny_full(), params.width, params.height)
    ref, _, st = gpu.render(scene, replace(params, shard_map=F.RP_SHARD_INTERLEAVE))
    plans = np.load(tmp_path / "plans.npy")
    assert (plans == plans[0]).all() and not np.array_equal(plans[0], np.arange(plans.shape[1]))
    assert np.array_equal(np.load(tmp_path / "frame.npy"), ref)
    assert int(np.load(tmp_path / "rays.npy")[0]) == st["rays"]
    rgba = np.zeros((params.width * params.height, 4), dtype=np.uint8)
    F.host().rph_to_srgb_u8(np.ascontiguousarray(ref).ctypes.data, params.width * params.height, rgba.ctypes.data)
    assert np.array_equal(np.load(tmp_path / "frame8.npy").reshape(-1, 4), rgba[:, [2, 1, 0, 3]])


def _frames_worker(rank, world, port, result_dir, n_frames):
    """A launch of n_frames frames of this rank's balanced shard, packed (rp_frames_pack), the packed blocks all-gathered
    over gloo in place of RCCL, and unpacked (rp_frames_unpack) into the n_frames assembled BGRA8 frames + summed
    counters on every rank."""
    import ctypes
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "raytracing-potato_amd")]
    import torch
    import torch.distributed as dist
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import shard_params
    from rtpotato.render import DeviceScene
    from rtpotato.scene import shard_slot_count
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    params = _frames_params()
    scene = scenes.configure(scenes.bunny_full(), params.width, params.height)
    sp = shard_params(params, rank, world)
    n = shard_slot_count(sp)
    pc = sp.to_c()
    words = ctypes.c_uint64()
    F.check(F.rp().rp_frames_block_words(ctypes.byref(pc), n_frames, ctypes.byref(words)))
    with DeviceScene(scene, device=0) as ds:
        ws = ds.workspace()
        ds.reserve_frames(sp, n_frames, ws)
        rgb = torch.zeros(3 * n * n_frames, dtype=torch.float64, device="cuda")
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        ds.render_frames_device(sp, n_frames, rgb, ctr, workspace=ws)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        send = torch.zeros(words.value, dtype=torch.int32, device="cuda")
        F.check(F.rp().rp_frames_pack(ds.handle, ws.handle, ctypes.byref(pc), n_frames, rgb.data_ptr(), ctr.data_ptr(),
                                      send.data_ptr(), st))
        torch.cuda.synchronize()
        blocks = [torch.zeros(words.value, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(blocks, send.cpu())
        recv = torch.cat(blocks).cuda()
        frames = torch.zeros(n_frames * params.width * params.height, dtype=torch.int32, device="cuda")
        total = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        F.check(F.rp().rp_frames_unpack(ds.handle, ws.handle, ctypes.byref(pc), n_frames, recv.data_ptr(),
                                        frames.data_ptr(), total.data_ptr(), st))
        torch.cuda.synchronize()
        np.save(os.path.join(result_dir, f"frames{rank}.npy"), frames.cpu().numpy().view(np.uint8))
        np.save(os.path.join(result_dir, f"ctr{rank}.npy"), total.cpu().numpy())
        np.save(os.path.join(result_dir, f"own{rank}.npy"), ctr.cpu().numpy())
        ws.close()
    dist.destroy_process_group()


def _frames_params():
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    return RenderParams(88, 56, 12, 8, scenes.DEFAULT_SEED, 16, 16, samples_per_stream=5, shard_map=F.RP_SHARD_BALANCED)


def test_two_process_frames_pack_unpack(gpu, tmp_path):
    """the multi-rank, multi-frame layout of rp_frames_gather's packed block -- rank blocks `words` apart,
    frame f's bytes at a fixed offset per frame, the counter reduce stepping over whole blocks -- exercised with two
    ranks (two processes on the box's one GPU, gloo in place of RCCL, which cannot put two ranks on one device): every
    rank's assembled frame f equals the one-process render of frame f (seed + f B W H) after to_srgb_u8, byte for
    byte, and the counters are the sums over the ranks' launches (each the sum of its frames)."""
    from dataclasses import replace
    from rtpotato import _ffi as F
    from rtpotato import scenes
    world, n_frames = 2, 3
    mp.spawn(_frames_worker, args=(world, _free_port(), str(tmp_path), n_frames), nprocs=world, join=True)
    params = _frames_params()
    scene = scenes.configure(scenes.bunny_full(), params.width, params.height)
    B = -(-params.spp // params.samples_per_stream)
    W, H = params.width, params.height
    own = sum(np.load(tmp_path / f"own{r}.npy") for r in range(world))
    rays = 0
    for f in range(n_frames):
        ref, _, st = gpu.render(scene, replace(params, shard_map=F.RP_SHARD_INTERLEAVE, seed=params.seed + f * B * W * H))
        rays += st["rays"]
        rgba = np.zeros((W * H, 4), dtype=np.uint8)
        F.host().rph_to_srgb_u8(np.ascontiguousarray(ref).ctypes.data, W * H, rgba.ctypes.data)
        for r in range(world):
            got = np.load(tmp_path / f"frames{r}.npy").reshape(n_frames, W * H, 4)[f]
            assert np.array_equal(got, rgba[:, [2, 1, 0, 3]]), (f, r)
    for r in range(world):
        c = np.load(tmp_path / f"ctr{r}.npy")
        assert c[:3].tolist() == own[:3].tolist() and c[3] == 0, (r, c, own)
    assert own[0] == rays and own[2] == n_frames * W * H

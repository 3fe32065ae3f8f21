"""The C-ABI libraries load on a CPU-only host and export every function their headers declare.
(No compute call: librp.so needs a gfx950 device for that; rp_device_count must still answer.)"""
import ctypes
import os
import re
import subprocess

from conftest import PKG, REPO


def _declared(header):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rph?_[a-z0-9_]+)\s*\(", src)))


def _exports(lib):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_librp_exports_all_rp_h_symbols():
    lib = os.path.join(PKG, "lib", "librp.so")
    names = _declared("rp.h")
    assert "rp_render" in names and "rp_render_device" in names and len(names) >= 11
    missing = set(names) - _exports(lib)
    assert not missing, missing
    from rtpotato import _ffi as F
    assert set(F.RP_SYMBOLS) == set(names)


def test_librp_host_exports_all_rp_host_h_symbols():
    lib = os.path.join(PKG, "lib", "librp_host.so")
    names = _declared("rp_host.h")
    missing = set(names) - _exports(lib)
    assert not missing, missing
    from rtpotato import _ffi as F
    assert set(F.HOST_SYMBOLS) == set(names)


def test_librp_loads_and_reports_without_gpu():
    from rtpotato import _ffi as F
    L = F.rp()
    assert L.rp_abi_version() == F.RP_ABI_VERSION == 9
    n = ctypes.c_int(-1)
    rc = L.rp_device_count(ctypes.byref(n))
    assert rc in (F.RP_OK, F.RP_ENODEV) and n.value >= 0


def test_struct_layouts_match_c():
    """ctypes mirrors of rp.h structs have the C sizes (checked against a tiny C program)."""
    import subprocess
    import tempfile
    from rtpotato import _ffi as F
    code = r'''
#include <stdio.h>
#include "rp.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %d %d %d\n", sizeof(rp_hittable), sizeof(rp_mesh), sizeof(rp_material),
         sizeof(rp_texture), sizeof(rp_scene_desc), sizeof(rp_camera), sizeof(rp_render_params), sizeof(rp_stats),
         sizeof(rp_scene_options), RP_COUNTERS_LEN, RP_SAMPLES_PER_STREAM, RP_COMM_ID_BYTES);
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(code)
        exe = os.path.join(d, "s")
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        sizes = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    ours = [ctypes.sizeof(t) for t in (F.rp_hittable, F.rp_mesh, F.rp_material, F.rp_texture, F.rp_scene_desc,
                                        F.rp_camera, F.rp_render_params, F.rp_stats, F.rp_scene_options)]
    assert sizes == ours + [F.RP_COUNTERS_LEN, F.RP_SAMPLES_PER_STREAM, F.RP_COMM_ID_BYTES]
    assert F.hittable_dtype().itemsize == ctypes.sizeof(F.rp_hittable)


def test_integration_rust_mirror_matches_c():
    """INTEGRATION.md's Rust #[repr(C)] mirrors of rp_render_params and rp_scene_options list the C fields in order
    (a missing trailing field would make the library read past the caller's struct)."""
    import re
    from rtpotato import _ffi as F
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    for rust, c in (("RpRenderParams", F.rp_render_params), ("RpSceneOptions", F.rp_scene_options)):
        body = re.search(r"pub struct " + rust + r" \{(.*?)\}", text, re.S).group(1)
        assert re.findall(r"pub (\w+):", body) == [f[0] for f in c._fields_], rust
        # the worked examples' struct literals name only real fields (a stale name would not compile)
        for lit in re.findall(r"\b" + rust + r" \{([^}]*)\}", text):
            if "pub " in lit:
                continue
            names = re.findall(r"(\w+)\s*:", lit)
            assert set(names) <= {f[0] for f in c._fields_}, (rust, names)


def test_no_oracle_in_product():
    """The product (librp.so, the package) never links or imports the oracle."""
    import subprocess
    for lib in ("librp.so", "librp_host.so"):
        out = subprocess.run(["ldd", os.path.join(PKG, "lib", lib)], capture_output=True, text=True).stdout
        assert "oracle" not in out
    for root, _, files in os.walk(os.path.join(PKG, "rtpotato")):
        for f in files:
            if f.endswith(".py"):
                assert "oracle" not in open(os.path.join(root, f)).read().replace("no oracle", "")


def test_scene_options_defaults_without_gpu():
    """rp_scene_options_init is host-only: the documented defaults."""
    from rtpotato.render import scene_options
    o = scene_options()
    assert (o.builder, o.max_leaf, o.cost_traverse, o.always_max, o.lds_depth, o.trav_threshold, o.tile_order,
            o.probe_n) == (0, 4, 0.7, 4, 0, 0, 0, 16)
    assert o.node_format == 0  # RP_NODES_AUTO: q8 for host trees of >= 2^21 hittables, f32 otherwise
    assert o.leaf_break == 0   # auto: 8 for cache-resident scenes, 16 above 256 MB
    assert o.unit_queues == 0 and o.queue_chunk == 0  # RP_QUEUES_AUTO: per-XCD queues; 0: chunks of 8 tiles
    assert o.collapse == 0  # RP_COLLAPSE_AUTO: the SAH-optimal 4-wide collapse
    o = scene_options(builder="gpu", lds_depth=17, node_format="q8")
    assert o.builder == 2 and o.lds_depth == 17 and o.node_format == 2


def test_product_library_reads_no_environment():
    """Every knob is an argument: librp.so's sources call no getenv (env vars changed results)."""
    import glob
    for f in glob.glob(os.path.join(PKG, "csrc", "*")):
        assert "getenv" not in open(f).read(), f


def test_product_kernel_refuses_result_changing_macros():
    """A build of the product kernel with a timing ablation (wrong streams or colours) is refused."""
    import subprocess
    src = os.path.join(PKG, "csrc", "rp_kernel.hip")
    for macro in ("RPK_ABLATE_RNG", "RPK_ABLATE_TEX", "RPK_BATCH_LEAF"):
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-E", f"-D{macro}", src, "-o", os.devnull],
                           capture_output=True, text=True)
        assert r.returncode != 0 and "result-changing" in r.stderr, macro


def test_product_kernel_has_no_experiment_switches():
    """The product kernel sources are the product path plus the RPK_DIAG instrumentation only:
    no #if on an experiment macro, and the switches of earlier rounds are refused by #error."""
    import subprocess
    allowed = {"RPK_DIAG", "RPK_DIAG_NOSTAMP", "RPK_DIAG_BIN_TICKS"}
    for f in ("rp_device.h", "rp_kernel.hip", "rp_kernel.h", "rp_layout.h"):
        src = open(os.path.join(PKG, "csrc", f)).read()
        conds = re.findall(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b(.*)$", src, flags=re.M)
        used = set()
        for c in conds:
            if "#error" in c:
                continue
            used |= set(re.findall(r"\bRPK_[A-Z0-9_]+", c))
        # the refusal list itself is a single #if feeding an #error
        refusal = set(re.findall(r"defined\((RPK_[A-Z0-9_]+)\)", src))
        assert used - allowed <= refusal, (f, used - allowed - refusal)
    src = os.path.join(PKG, "csrc", "rp_kernel.hip")
    for macro in ("RPK_NT_STORE", "RPK_COLD_IN_SLAB", "RPK_NO_SPECULATIVE", "RPK_TRIES=3"):
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-E", f"-D{macro}", src, "-o", os.devnull],
                           capture_output=True, text=True)
        assert r.returncode != 0 and "experiment macros" in r.stderr, macro


def test_profile_records_are_of_this_build():
    """bench.py prices its roofline with the per-ray records profiles/current.json names and refuses a record of
    another build; the committed records must be the ones of the kernel the committed sources build (rp_build_id
    hashes the render kernel's code object), so a kernel change cannot ship with stale records."""
    import json
    from rtpotato import _ffi as F
    build = F.rp().rp_build_id().decode()
    cur = json.load(open(os.path.join(REPO, "profiles", "current.json")))["roofline"]
    # keys "<config>" or "<config>@<samples_per_stream>" (bench.py kernel_record): the N = 1 headline's C3 record under
    # the one-stream contract, the 32-sample streams N > 1 runs use, and C5
    assert "C3" in cur and "C3@32" in cur and any(k.split("@")[0] == "C5" for k in cur)
    for key, rel in cur.items():
        rec = json.load(open(os.path.join(REPO, rel)))
        cfg, _, sps = key.partition("@")
        assert rec["build_id"] == build, (key, rel, rec["build_id"], build)
        assert rec["config"] == cfg and rec["rays"] > 0 and rec["traffic_bytes_per_ray"] > 0
        assert not sps or rec["samples_per_stream"] == int(sps), (key, rec.get("samples_per_stream"))
    assert json.load(open(os.path.join(REPO, cur["C3"])))["samples_per_stream"] == 256


def test_build_id_is_path_independent(tmp_path):
    """rp_build_id must not depend on the directory the library is built in (a clean checkout elsewhere
    must keep the committed records valid).  The same HIP source compiled at two paths gives objects whose whole
    .hip_fatbin differs (a path-derived __hip_cuid symbol) but whose build_id.sh hash -- the one the Makefile stamps --
    is the same."""
    import hashlib
    src = ("#include <hip/hip_runtime.h>\n__global__ void k(float* x) { x[threadIdx.x] *= 2.0f; }\n"
           "void run(float* x, hipStream_t s) { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, x); }\n")
    ids, fats = [], []
    for sub in ("a", "bb/longer_path"):
        d = tmp_path / sub
        d.mkdir(parents=True)
        (d / "t.hip").write_text(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-fPIC", "-c", str(d / "t.hip"), "-o", "t.o"],
                       cwd=d, check=True, capture_output=True)
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", "t.o", "fat.bin"], cwd=d, check=True)
        fats.append(hashlib.sha256((d / "fat.bin").read_bytes()).hexdigest())
        r = subprocess.run(["bash", os.path.join(PKG, "build_id.sh"), "gfx950", str(d / "t.o"), "--", str(d / "t.o")],
                           capture_output=True, text=True, check=True)
        ids.append(r.stdout.strip())
    assert len(ids[0]) == 16 and ids[0] == ids[1], ids
    assert fats[0] != fats[1]  # what the round-4 id hashed


def test_bench_cpu_fit_is_a_least_squares_line():
    """bench.py's full-host CPU figure is a least-squares line through >= 3 measured worker counts,
    not a two-point ratio: exact on collinear points, and its R^2 shows a bend."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    lin = b.fit_workers([{"workers": w, "value": 0.5 + 0.9 * w} for w in (1, 4, 8, 16)])
    assert abs(lin["intercept"] - 0.5) < 1e-9 and abs(lin["per_worker"] - 0.9) < 1e-9 and lin["r2"] == 1.0
    bent = b.fit_workers([{"workers": w, "value": v} for w, v in ((1, 1.0), (4, 4.0), (8, 7.0), (16, 11.0))])
    assert bent["per_worker"] < 0.75 and bent["r2"] < 1.0 and bent["points"] == 4


def test_profile_records_price_fractions_below_one():
    """the bench line's fractions are of a roof -- priced at the record's own frame time, the memory-side
    traffic is <= 8 TB/s (roofline.frac), the algorithmic bytes <= the L2 gather rate (roofline.l2_level) and the VALU
    issue <= 1 (binding_frac)."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    cur = json.load(open(os.path.join(REPO, "profiles", "current.json")))["roofline"]
    for cfg, rel in cur.items():
        rec = json.load(open(os.path.join(REPO, rel)))
        secs = rec["bench_ms_per_step"] / 1e3  # per frame
        rate = rec["rays"] / sum(rec.get("frames_per_launch", [1])) / secs
        assert 0 < rec["traffic_bytes_per_ray"] * rate / 1e9 / b.HBM_PEAK_GBS <= 1.0, cfg
        assert 0 < rec["algorithmic_bytes_per_ray"] * rate / 1e9 / b.L2_GATHER_GBS <= 1.0, cfg
        assert 0 < rec["valu_per_ray"] * rate / b.VALU_ISSUE_PEAK <= 1.0, cfg


def test_bench_launch_sizes():
    """bench.py splits K frames into the fewest launches of <= L frames, sizes near-equal (the driver's --steps 20 at
    8 per launch: 7 + 7 + 6), and spreads the warm-up over the in-flight workspaces."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.launch_sizes(20, 8) == [7, 7, 6]
    assert b.launch_sizes(20, 32) == [20] and b.launch_sizes(20, 16) == [10, 10]  # the driver's 20 steps at L = 32 / 16
    assert b.launch_sizes(16, 8) == [8, 8] and b.launch_sizes(8, 8) == [8] and b.launch_sizes(5, 8) == [5]
    assert b.launch_sizes(0, 8) == [] and b.launch_sizes(3, 1) == [1, 1, 1]
    assert b.launch_sizes(5, 8, 3) == [2, 2, 1] and b.launch_sizes(2, 8, 2) == [1, 1]
    for n in range(1, 70):
        for L in (1, 3, 8, 16):
            s = b.launch_sizes(n, L)
            assert sum(s) == n and max(s) <= L and max(s) - min(s) <= 1 and len(s) == -(-n // L)


def test_bench_frames_per_launch_cap():
    """bench.py keeps a launch's units below 2^31 (rp_api.cpp refuses more): C3 takes its 16 frames, C5 15, C4 (1,024 spp,
    32 batches) 16 of its 32 allowed."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    c3 = 60 * 34 * 1024  # 32 x 32 tiles of a 1920 x 1080 frame
    assert b.frames_per_launch_cap(16, c3, 8) == 16 and b.frames_per_launch_cap(64, c3, 32) == 32
    c5 = 128 * 128 * 1024
    assert b.frames_per_launch_cap(16, c5, 8) == 15 and b.frames_per_launch_cap(16, c5, 8) * c5 * 8 < 1 << 31
    assert b.frames_per_launch_cap(1, 0, 0) == 1 and b.frames_per_launch_cap(8, 1 << 31, 1) == 1
    # the library's per-XCD queue bound, 2 n + lanes < 2^32 - 1, is the binding one (it is below 2^31)
    for slots, batches in ((c3, 1), (c3, 8), (c5, 8), (1 << 20, 3), ((1 << 31) // 2 - 1000, 1)):
        for lanes in (262_144, b.LANES_MAX):
            L = b.frames_per_launch_cap(64, slots, batches, lanes)
            n = slots * batches * L
            assert L == 1 or (n < 1 << 31 and 2 * n + lanes < 0xFFFFFFFF), (slots, batches, lanes, L)
            assert L == 64 or 2 * (n + slots * batches) + lanes >= 0xFFFFFFFF - 1 or (n + slots * batches) >= 1 << 31


def test_bench_frame_sequence_seeds():
    """bench.py's launches take consecutive frames of one sequence, so the warm-up's frames and the timed
    frames (and the single-frame and side-leg frames after them) have disjoint seeds -- for every per-pixel stream, since
    frame f's stream of (pixel, batch) is seed + f B W H + b W H + j W + i."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    W, H, seed = 1920, 1080, 1592590337
    for nb, warm, steps, L in ((1, 5, 20, 32), (8, 5, 20, 32), (8, 8, 16, 8), (1, 3, 7, 1)):
        seq = b.FrameSeq()
        phases = []
        for sizes in (b.launch_sizes(warm, L), b.launch_sizes(steps, L), [1, 1, 1]):
            streams = set()
            for n in sizes:
                f0, s0 = seq.launch(seed, nb, W, H, n)
                assert s0 == b.frame_seed(seed, nb, W, H, f0)
                for f in range(n):  # frame f of the launch: s0 + f B W H (rp_render_frames_device_ws)
                    fs = (s0 + f * nb * W * H) & b.U64
                    streams.add(fs)
            phases.append(streams)
        assert len(phases[0]) == warm and len(phases[1]) == steps
        assert not (phases[0] & phases[1]) and not (phases[1] & phases[2]) and not (phases[0] & phases[2])
        # a frame's per-pixel streams occupy [fs, fs + B W H): consecutive frames never share one
        allf = sorted(phases[0] | phases[1] | phases[2])
        assert all(y - x >= nb * W * H for x, y in zip(allf, allf[1:]))
    assert b.frame_seed(b.U64, 1, 1, 1, 1) == 0  # u64 wrap, like rp_render_params.seed

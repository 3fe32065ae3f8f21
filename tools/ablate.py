"""Timing-only A/B: C3 64-spp frame time per variant, interleaved rounds.  A variant is a library file
under raytracing-potato_amd/lib, optionally with a traversal threshold and rp_scene_options fields:
`librp.so@16` (trav_threshold), `librp.so@40:max_leaf=2,cost_traverse=1.5`."""
import os, sys, json, subprocess
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:]
res = {}
for rnd in range(2):
    for spec in libs:
        # spec: LIB[@THRESHOLD][:ENV=VALUE,...]
        head, _, extra = spec.partition(":")
        lib, _, thr = head.partition("@")
        env = dict(os.environ)
        opts = {}
        if thr:
            opts["trav_threshold"] = int(thr)
        for kv in filter(None, extra.split(",")):
            k, _, v = kv.partition("=")
            opts[k] = float(v) if "." in v else (v if k == "builder" else int(v))
        code = f"""
import os,sys
sys.path[:0]=['{REPO}','{REPO}/raytracing-potato_amd']
os.environ['RP_LIB']='{REPO}/raytracing-potato_amd/lib/{lib}'
from dataclasses import replace
from rtpotato import scenes
from rtpotato.render import DeviceScene
sc,p=scenes.config_scene("C3"); p=replace(p, spp=int(os.environ.get("ABLATE_SPP","64")))
ds=DeviceScene(sc, options={opts!r}); ds.render(replace(p,spp=4))
ts=[ds.render(p)[2]['seconds'] for _ in range(2)]
print(min(ts))
"""
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        res.setdefault(spec, []).append(float(out.stdout.strip().split()[-1]) if out.returncode == 0 else out.stderr[-300:])
print(json.dumps(res))

"""Quick check of the device builders (diagnostic): the same image and ray count from the host SAH, LBVH and PLOC trees (with the structural self-check), and the oracle's."""
import sys, time
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, os.path.join(R, 'raytracing-potato_amd'), os.path.join(R, 'tests')]
import numpy as np
from dataclasses import replace
from rtpotato import scenes
from rtpotato.render import DeviceScene
from parity import oracle_render, compare
sc = scenes.configure(scenes.bunny_full(), 96, 64)
from rtpotato.scene import RenderParams
p = RenderParams(96, 64, 8, 8, scenes.DEFAULT_SEED)
for b in ("host", "gpu", "ploc"):
    with DeviceScene(sc, options={"builder": b, "self_check": 1}) as ds:
        rgb, _, st = ds.render(p)
        print(b, ds.info(), st["rays"], flush=True)
ref, _, ctr = oracle_render(sc, p, threads=8)
print("oracle rays", ctr["rays"], compare(rgb, ref))

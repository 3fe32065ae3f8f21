"""Regenerate the packed asset fixtures from the reference's asset files (run where /root/reference exists).

    python raytracing-potato_amd/assets/make_assets.py

bunny.npz / bunny_flat.npz: obj::load (mesh.rs:145-183) output of assets/bunny.obj / bunny_flat.obj.
earthmap.npz: tga::load (image.rs:73-114) output of assets/earthmap.tga (RGBA8, row 0 = bottom).
Both go through librp_host.so's loaders; tests/test_host.py checks the fixtures against a fresh load.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from rtpotato import assets  # noqa: E402


def main():
    ref = assets.REFERENCE_ASSETS
    for name in ("bunny", "bunny_flat"):
        m = assets.obj_load(os.path.join(ref, name + ".obj"))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), positions=m.positions, normals=m.normals,
                            uvs=m.uvs, indices=m.indices)
        print(name, m.positions.shape, m.indices.shape)
    img = assets.tga_load(os.path.join(ref, "earthmap.tga"))
    np.savez_compressed(os.path.join(HERE, "earthmap.npz"), rgba=img)
    print("earthmap", img.shape)


if __name__ == "__main__":
    main()

"""The bounce-0 dielectric-reflect path, which a gfx950 code-generation problem once broke.

With the primary ray's throughput T a compile-time (1, 1, 1), ROCm 7.2 clang dropped T.xy on the
dielectric-reflect path of scatter() (scene.cu:443-476) inside the shade kernel; shade_one launders
T through an empty asm at bounce 0 (csrc/rt_render.hip).  Two checks:
* tests/native/miscompile_repro: the same scatter() in a standalone kernel, T constant vs laundered,
  against the host build of the same source -- the laundered form must match bit for bit; the JSON
  records whether this standalone shape reproduces the problem;
* renders of a glass sphere filling the view, 2-3 bounces, sort on and off, against the oracle: every
  primary ray takes the dielectric branch at bounce 0 and its T reaches the image through the sky
  lookup of bounce 1, so a dropped T.xy changes the image."""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

GLASS = ("material glass ior 1.5 roughness 0 specular 0.9 0.8 0.7 diffuse 0.95 0.9 0.85\n"
         "material floor diffuse 0.5 0.5 0.5\n"
         "sphere glass 0 0 0 1\n"
         "quad floor -20 -1 -20 -20 -1 20 20 -1 20 20 -1 -20\n"
         "sky 0.6 0.7 0.9\n"
         "camera position 0 0.2 -2.6 forward 0 -0.05 1 up 0 1 0 fov 50\n"
         "image 64 48 20 3 1\n")


def test_standalone_scatter_laundered_matches_host():
    exe = os.path.join(HERE, "native", "build", "miscompile_repro")
    assert os.path.exists(exe), "tests/native not built (__graft_entry__.build())"
    out = subprocess.run([exe, "65536"], capture_output=True, text=True, timeout=120, check=True).stdout
    rec = json.loads(out.strip().splitlines()[-1])
    print("miscompile_repro:", rec)
    assert rec["dielectric_reflect"] > 1000
    assert rec["laundered_mismatch"] == 0


@pytest.mark.parametrize("bounces,sort", [(2, True), (2, False), (3, True)])
def test_glass_sphere_first_bounce_bitexact(tmp_path, bounces, sort):
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    path = str(tmp_path / "glass.scene")
    with open(path, "w") as f:
        f.write(GLASS)
    image = (64, 48, 20, bounces)
    ofb, ost = O.OracleScene(path, image=image).render(sort=sort)
    gfb, gst = R.render(R.Scene(path, image=image), sort=sort, counters=True)
    assert np.array_equal(gfb, ofb)
    assert gst["hits_sphere"] == ost["hits_sphere"] and gst["hits_sphere"] > 64 * 48 * 20 // 4

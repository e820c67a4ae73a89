"""Synthetic scene files that drive traversal paths the shipped scenes reach rarely or never.

* big_leaf: 80 triangles with one common centroid (rotated copies).  The binned SAH split
  (scene.cu:866-1000) finds min_centroid == max_centroid on every axis, so they end in one leaf
  of 80 triangles: the renderer's leaf refs hold at most 63 inline, larger leaves go through the
  indirection table.
* deep: 60 triangles at x = 3^k.  The binned split peels off the farthest triangle at every
  level, so the tree is a chain as deep as MAX_BVH_DEPTH (30, scene.cu:10) allows.  A ray
  coming from +x enters each level's single-triangle child first, so the reference pushes that
  near child and descends into the far subtree: the stack grows by one per level, past the
  8 entries the trace kernel keeps in LDS into its global overflow.  The triangles' yz
  projections box the x axis without covering it, so rays along the axis hit nothing and walk
  the whole chain.
"""
import math
import os


def _tri(p, q, r):
    return "triangle white %s %s %s\n" % tuple(" ".join("%.9g" % c for c in v) for v in (p, q, r))


DEEP_COUNT, DEEP_RATIO = 60, 3.0   # a 30-level chain (59 nodes): one triangle split off per level

HEADER = ("material white diffuse 0.8 0.8 0.8 metallicity 0.2 specular 1 1 1 roughness 0.3\n"
          "material grey diffuse 0.5 0.5 0.5\n"
          "sky 0.6 0.7 0.9\n")


def big_leaf_scene():
    s = HEADER
    for k in range(80):
        a = 2 * math.pi * k / 80
        dx, dz = 0.5 * math.cos(a), 0.5 * math.sin(a)
        # p and q mirror each other about the y axis (their printed x and z negate exactly) and
        # r = (0, 0, 0): the float centroid of every triangle is exactly (0, 1, 0)
        s += _tri((dx, 1.5, dz), (-dx, 1.5, -dz), (0.0, 0.0, 0.0))
    s += "quad grey -20 0 -20 -20 0 20 20 0 20 20 0 -20\n"
    s += "camera position -4 1.5 0 forward 1 -0.1 0 up 0 1 0 fov 40\n"
    s += "image 48 32 20 4 1\n"
    return s


def deep_scene():
    s = HEADER
    for k in range(DEEP_COUNT):
        x = DEEP_RATIO ** k
        # yz projection (-1, 1.2), (1, 1), (1.2, -1): its box holds (0, 0), the triangle does not
        s += _tri((x, -1.0, 1.2), (x + 0.01, 1.0, 1.0), (x + 0.02, 1.2, -1.0))
    s += "camera position 1e29 0.05 0.05 forward -1 0 0 up 0 1 0 fov 2\n"
    s += "image 32 32 20 3 1\n"
    return s


def write(dirpath):
    """Writes big_leaf.scene and deep.scene into dirpath; returns their paths."""
    out = {}
    for name, text in (("big_leaf", big_leaf_scene()), ("deep", deep_scene())):
        p = os.path.join(dirpath, name + ".scene")
        with open(p, "w") as f:
            f.write(text)
        out[name] = p
    return out

"""The closed form of the reference's two-pointer partition (scene.cu:960-975) that the GPU BVH
build uses (csrc/bvh_build.hip, partition_kernel), checked here against the loop itself on
random and adversarial left/right patterns.  No GPU: this pins the algebra the kernel runs."""
import numpy as np
import pytest


def loop_partition(left):
    """The reference's loop on element ids 0..n-1: returns the final order and the split index."""
    a = list(range(len(left)))
    i, j = 0, len(a) - 1
    while i <= j:
        if left[a[i]]:
            i += 1
        else:
            a[i], a[j] = a[j], a[i]
            j -= 1
    return a, i


def closed_form(left):
    """partition_kernel's destinations, phase by phase."""
    n = len(left)
    L = int(sum(left))
    a = L if (L == n or left[L]) else L + 1
    X, R = {}, {}
    dest = [None] * n
    k = 0
    for p in range(a):                       # front: rights get rank k, X[k] = position
        if not left[p]:
            X[k] = p
            k += 1
    kl = kr = 0
    for y in range(n - a):                   # back, descending positions
        p = n - 1 - y
        if left[p]:
            R[kl] = kr
            kl += 1
        else:
            dest[p] = n - 1 - (kl + 1 + kr)
            kr += 1
    kl = 0
    for y in range(n - a):
        p = n - 1 - y
        if left[p]:
            dest[p] = X[kl]
            kl += 1
    k = 0
    for p in range(a):
        if left[p]:
            dest[p] = p
        else:
            dest[p] = n - 1 - (k + (R[k - 1] if k >= 1 else 0))
            k += 1
    order = [None] * n
    for src, d in enumerate(dest):
        assert order[d] is None
        order[d] = src
    return order, L


@pytest.mark.parametrize("seed", range(200))
def test_closed_form_equals_loop_random(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 80))
    left = list(rng.random(n) < rng.random())
    assert closed_form(left) == loop_partition(left)


def test_closed_form_equals_loop_exhaustive_small():
    for n in range(1, 13):
        for bits in range(1 << n):
            left = [(bits >> k) & 1 == 1 for k in range(n)]
            assert closed_form(left) == loop_partition(left), left

"""Host restatement of the interleaved-payload layout (bucket_sort.hpp,
k_interleave): the scan-free row-block bases computed from the schedule's
class totals must equal the direct prefix sum over the wave groups' heads,
blocks must not overlap, and the array must fit ne + BS_IPAY_SLACK entries.
(CPU only; the GPU path is covered by the parity tests, e.g.
test_gpu_ches.py::test_skewed_buckets_mixed_payload_layout.)"""
import random

import pytest

SLACK = 64 * 256


def sched_class(c):
    return 255 - min(c, 255)


def kernel_bases(counts):
    """k_interleave's arithmetic: class totals -> ct, heads per class -> hs,
    then per wave group the class of its head position and its base."""
    nb = len(counts)
    tot = [0] * 256
    for c in counts:
        tot[sched_class(c)] += 1
    ct = [0] * 256
    for c in range(1, 256):
        ct[c] = ct[c - 1] + tot[c - 1]
    t0r = (ct[1] + 63) & ~63
    contrib = []
    for c in range(256):
        lo, hi = max(ct[c], t0r), ct[c] + tot[c]
        contrib.append((255 - c) * (((hi + 63) >> 6) - ((lo + 63) >> 6)) if c > 0 and lo < hi else 0)
    hs = [0] * 256
    for c in range(1, 256):
        hs[c] = hs[c - 1] + contrib[c - 1]
    nw = (nb + 63) // 64
    bases = []
    for g in range(nw):
        head = g << 6
        if head < t0r or head >= nb:
            bases.append(None)
            continue
        c = 0
        step = 128
        while step:
            if ct[c + step] <= head:
                c += step
            step >>= 1
        first = max(ct[c], t0r)
        bases.append(hs[c] + (255 - c) * ((head >> 6) - ((first + 63) >> 6)))
    return bases


def schedule(counts, rnd):
    """positions by class (k_sched_scatter: classes ascending, any order within)"""
    order = list(range(len(counts)))
    rnd.shuffle(order)
    order.sort(key=lambda b: sched_class(counts[b]))
    return [counts[b] for b in order]


@pytest.mark.parametrize("case", ["poisson13", "heavy", "sparse", "all_equal", "tiny", "skewed"])
def test_interleave_bases_match_prefix_of_heads(case):
    rnd = random.Random(hash(case) & 0xffff)
    nb = {"tiny": 70, "sparse": 5000}.get(case, 20000)
    if case == "poisson13":
        counts = [sum(rnd.random() < 13 / 40 for _ in range(40)) for _ in range(nb)]
    elif case == "heavy":  # a few buckets past 255 (class 0), the rest ordinary
        counts = [rnd.randrange(0, 30) for _ in range(nb)]
        for b in rnd.sample(range(nb), 37):
            counts[b] = rnd.randrange(255, 5000)
    elif case == "sparse":
        counts = [1 if rnd.random() < 0.05 else 0 for _ in range(nb)]
    elif case == "all_equal":
        counts = [0] * nb
        counts[5] = 1 << 16
    elif case == "tiny":
        counts = [rnd.randrange(0, 300) for _ in range(nb)]
    else:
        counts = [int(rnd.paretovariate(1.2)) for _ in range(nb)]
    sc = schedule(counts, rnd)
    ne = sum(counts)
    bases = kernel_bases(counts)
    nxt = 0
    used = []
    for g, b in enumerate(bases):
        grp = sc[64 * g:64 * g + 64]
        if b is None:
            # only groups starting inside class 0 (or none at all) fall back
            assert 64 * g < ((sum(1 for c in counts if c >= 255) + 63) & ~63) or not grp
            continue
        head = grp[0]
        assert head == max(grp) and head < 255
        assert b == nxt, g  # = the direct prefix sum over the heads of earlier interleaved groups
        used.append((b, b + head))
        nxt += head
    assert nxt * 64 <= ne + SLACK  # fits the per-set stride

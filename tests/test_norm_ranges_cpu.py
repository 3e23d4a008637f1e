"""The fused grad-norm bookkeeping (train/optimizer.py): the norm chunks skip the flat ranges whose Σg²
the grouped weight-gradient launch writes itself, keeping everything else exactly once."""

import random

from distributed_training_compare_jax_amd.train.optimizer import _subtract_ranges


def _cover(segs):
    out = set()
    for o, n, _ in segs:
        out.update(range(o, o + n))
    return out


def test_subtract_ranges_exact_cover():
    rng = random.Random(0)
    for _ in range(200):
        segs, o = [], 0
        for _ in range(rng.randint(1, 6)):
            o += rng.randint(0, 8)
            n = rng.randint(1, 40)
            segs.append((o, n, rng.choice([1.0, 0.5])))
            o += n
        ranges, r = [], 0
        for _ in range(rng.randint(0, 5)):
            r += rng.randint(0, 30)
            n = rng.randint(1, 30)
            ranges.append((r, n))
            r += n
        got = _subtract_ranges(segs, ranges)
        cut = set()
        for ro, rn in ranges:
            cut.update(range(ro, ro + rn))
        assert _cover(got) == _cover(segs) - cut
        # no overlaps, weights carried over
        assert sum(n for _, n, _ in got) == len(_cover(got))
        for go, gn, gw in got:
            src = [s for s in segs if s[0] <= go and go + gn <= s[0] + s[1]]
            assert len(src) == 1 and src[0][2] == gw

"""LDS layout of the fused attention backward (csrc/attention.hip, attn_bwd_fused_kernel): unpadded
[rows][32] bf16 panels with 16-B chunk c of row r stored at chunk c ^ fb_swz(r).

Checked on the CPU by simulating the gfx950 LDS banks (MI355X_MICROARCH.md §LDS: 64 banks of 4 B;
ds_read_b128 is serviced in four 16-lane groups, ds_read_b64 in two 32-lane groups) and by reading a
numbered panel through the swizzled addresses: every fragment must return the same elements as the
padded-row reads of the resident kernels (row_frag / tr_frag), and be bank-conflict-free.
"""

import numpy as np
import pytest

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
B64_GROUPS = [list(range(32)), list(range(32, 64))]


def fb_swz(r):
    return (0x1320 >> (((r >> 2) & 3) * 4)) & 3


def elem_off(r, col):
    """element offset of (row, hd column) in the swizzled panel"""
    return r * 32 + (((col >> 3) ^ fb_swz(r)) << 3) + (col & 7)


def fb_row_addrs(r0):
    """per lane: (element offset of the 8-element read, the 8 (row, col) it must hold)"""
    out = []
    for lane in range(64):
        r, c = r0 + (lane & 15), lane >> 4
        out.append((r * 32 + ((c ^ fb_swz(r)) << 3), [(r, 8 * c + e) for e in range(8)]))
    return out


def fb_tr_addrs(r0, t, second):
    """per lane: element offset of the 4-element (8-B) transposed read (p0, or p1 = +16 rows)"""
    out = []
    for lane in range(64):
        g, li = lane >> 4, lane & 15
        q, pp = li >> 2, li & 3
        r = r0 + 4 * g + q + (16 if second else 0)
        c = 2 * t + (pp >> 1)
        out.append(r * 32 + ((c ^ fb_swz(r)) << 3) + (pp & 1) * 4)
    return out


def conflicts(addr_bytes, width, groups):
    worst = 0
    for grp in groups:
        banks = []
        for lane in grp:
            a = addr_bytes[lane]
            banks += [((a // 4) + d) % 64 for d in range(width // 4)]
        worst = max(worst, len(banks) - len(set(banks)))
    return worst


@pytest.mark.parametrize("r0", [0, 16, 32, 48, 64, 496, 560])
def test_row_fragment_conflict_free_and_correct(r0):
    panel = np.full(600 * 32, -1)
    for r in range(600):
        for col in range(32):
            panel[elem_off(r, col)] = r * 32 + col
    reads = fb_row_addrs(r0)
    for off, want in reads:
        got = panel[off:off + 8]
        assert list(got) == [r * 32 + c for r, c in want]
    assert conflicts([2 * off for off, _ in reads], 16, B128_GROUPS) == 0


@pytest.mark.parametrize("r0", [0, 16, 32, 64, 480, 544])
@pytest.mark.parametrize("t", [0, 1])
def test_transposed_fragment_conflict_free_and_correct(r0, t):
    panel = np.full(600 * 32, -1)
    for r in range(600):
        for col in range(32):
            panel[elem_off(r, col)] = r * 32 + col
    for second in (False, True):
        offs = fb_tr_addrs(r0, t, second)
        # the padded-layout tr_frag reads row (r0 + 4g + q [+16]), columns 16t + 4pp .. +3
        for lane, off in enumerate(offs):
            g, li = lane >> 4, lane & 15
            q, pp = li >> 2, li & 3
            r = r0 + 4 * g + q + (16 if second else 0)
            assert list(panel[off:off + 4]) == [r * 32 + 16 * t + 4 * pp + e for e in range(4)]
        assert conflicts([2 * o for o in offs], 8, B64_GROUPS) == 0


def test_unswizzled_rows_would_conflict():
    """the check is sensitive: plain 64-B rows give 2-way conflicts on the row fragments"""
    addrs = [2 * ((lane & 15) * 32 + 8 * (lane >> 4)) for lane in range(64)]
    assert conflicts(addrs, 16, B128_GROUPS) > 0

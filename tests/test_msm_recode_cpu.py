"""CPU: the two-level MSM sort (msm.hip rs_point_digits, used by k_rs_hist /
k_rs_scatter) reads window w's signed digit of a GLV half k as a plain bit
field of k + C, C = sum_w (2^(width_w-1) - 1) 2^off_w.  Check that this gives
exactly k_msm_digits' sequential recoding (d = bits + carry; carry' = d > half;
d -= 2^width if carry') for the balanced window layouts msm_layout_groups
builds (device/msm.hpp), including the edge magnitudes."""
import random

import pytest

MSM_BITS = 127


def layout(c):
    nw = (MSM_BITS + c - 1) // c
    lo, extra = MSM_BITS // nw, MSM_BITS % nw
    wins, off = [], 0
    for w in range(nw):
        width = lo + (1 if w < extra else 0)
        wins.append((off, width))
        off += width
    return wins


def sequential(k, wins):
    out, carry = [], 0
    for off, width in wins:
        d = ((k >> off) & ((1 << width) - 1)) + carry
        half = 1 << (width - 1)
        carry = 1 if d > half else 0
        out.append(d - (1 << width) if carry else d)
    assert carry == 0
    return out


def bitfield(k, wins):
    C = sum(((1 << (width - 1)) - 1) << off for off, width in wins)
    kp = k + C
    assert kp < 1 << 127  # bit 127 holds the half's sign on the device
    return [((kp >> off) & ((1 << width) - 1)) - ((1 << (width - 1)) - 1) for off, width in wins]


@pytest.mark.parametrize("c", [5, 8, 11, 13, 15, 16])
def test_bitfield_digits_equal_sequential_recoding(c):
    wins = layout(c)
    rng = random.Random(c)
    ks = [0, 1, (1 << 126) - 1, 1 << 125] + [rng.getrandbits(126) for _ in range(3000)]
    # every window at its carry boundaries: fields of all-ones and of exactly half
    for off, width in wins:
        ks.append(((1 << width) - 1) << off)
        ks.append((1 << (width - 1)) << off)
        ks.append(((1 << (width - 1)) + 1) << off)
    for k in ks:
        k &= (1 << 126) - 1
        d = bitfield(k, wins)
        assert d == sequential(k, wins), (c, hex(k))
        assert sum(di << off for di, (off, _) in zip(d, wins)) == k

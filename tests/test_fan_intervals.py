"""The lean K-tick kernel's interval fans (csrc/heist_fan_intervals.h, heist_env.hip
`cast_ivl`), checked on CPU before any GPU run.

1. The table: tools/gen_fan_intervals.py's cuts recomputed here in float64 (acos / asin of
   the 31 tie points j/k, j odd, k <= 12, plus the axes) equal the header's to within 2
   units (2^32 units per turn); every interval's fp32 midpoint direction gives the same 12
   sample tiles (real-number rint) as points a margin inside both of its ends.
2. The partition: a Python restatement of the kernel's per-lane arithmetic (fixed-point
   camera angle, first ray above a cut, safe / near classification) turns a camera into
   {intervals to march} + {rays for the exact path}.  Marching the intervals' directions
   and casting the near rays as security.py:53-101 does, from the same tile over the same
   walls, gives exactly the oracle's cone (oracle/heist_oracle.c, pinned to the
   reference's golden cones) -- on random cameras, on headings whose rays sit on the axes
   (the reference's default camera: heading 0, fov 60) and on rays placed a few units from
   a cut.  The restatement is the kernel's specification: keep the two in step.
"""
import math
import os
import re

import numpy as np
import pytest

from oracle import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
HDR = os.path.join(os.path.dirname(HERE), "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd",
                   "csrc", "heist_fan_intervals.h")
U = 2 ** 32
UPD = 4294967296.0 / 360.0  # units per degree (heist_env.hip kFanUnitsPerDeg)


def _table():
    s = open(HDR).read()
    cut = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{8})u", s.split("kFanCut[kFanCuts] = {")[1].split("};")[0])]
    dirs = [(float.fromhex(a), float.fromhex(b)) for a, b in
            re.findall(r"\{([-0-9a-fx.p+]+)f, ([-0-9a-fx.p+]+)f\}", s.split("kFanDir[kFanCuts][2] = {")[1].split("};")[0])]
    idx = [int(x) for x in re.findall(r"\d+", s.split("kFanIdx[361] = {")[1].split("};")[0])]
    mt = int(re.search(r"kFanMarginTie = (\d+)", s).group(1))
    ma = int(re.search(r"kFanMarginAxis = (\d+)", s).group(1))
    return cut, dirs, idx, mt, ma


CUT, DIRS, IDX, MT, MA = _table()


def _offsets(dx, dy):
    return tuple((int(np.rint(k * dx)), int(np.rint(k * dy))) for k in range(1, 13))


def test_table_matches_float64_recomputation():
    ties = sorted({j / k for k in range(1, 13) for j in range(1, k, 2)})
    assert len(ties) == 31
    want = {0, U // 4, U // 2, 3 * U // 4}
    for t in ties:
        for b in (math.degrees(math.acos(t)), math.degrees(math.asin(t))):
            for a in (b, 180 - b, 180 + b, 360 - b):
                want.add(int(round(a * UPD)) % U)
    want = sorted(want)
    assert len(CUT) == len(want) == 252 and len(DIRS) == 252 and len(IDX) == 361
    assert max(abs(a - b) for a, b in zip(CUT, want)) <= 2
    assert all(CUT[i] < CUT[i + 1] for i in range(251))
    for j, c in enumerate(CUT):
        nxt = CUT[j + 1] if j + 1 < 252 else U
        m0 = MA if c % (U // 4) == 0 else MT
        m1 = MA if nxt % (U // 4) == 0 else MT
        w = _offsets(*DIRS[j])
        for a in (c + m0, nxt - m1):
            r = math.radians(a / UPD)
            assert _offsets(math.cos(r) / 2, -math.sin(r) / 2) == w, j
    for d in range(361):
        lim = -(-d * U // 360)
        assert IDX[d] == sum(1 for c in CUT if c < lim)


def fan_lanes(heading, fov):
    """The kernel's partition of one camera's rays (heist_env.hip step_lean_kernel cast_ivl, same
    arithmetic): returns (intervals to march, near ray indices for the exact path).  Ray i
    sits i * s units past h0; cut j (rel units past h0, margin m) owns rays ceil((rel - m) / s)
    .. floor((rel + m) / s) (exact path); interval j the rays after those up to the next cut's.
    The divisions are integer products: floor(x / s) = (mulhi(x, im) >> 20) with
    im = rint(2^52 / s) (v_mul_hi_i32, an arithmetic shift), ceil(x / s) = -floor(-x / s)."""
    n = max(int(fov * 2), 30)  # security.py:67
    hmh = heading - fov / 2.0
    hw = hmh + 360.0 if hmh < 0.0 else hmh
    h0 = int(min(hw * UPD, 4294967295.0))
    s = (fov / float(n)) * UPD
    assert s >= 2097153.0  # the kernel's eligibility: im fits an int32
    im = round(4503599627370496.0 / s)  # rint (ties to even, as round())
    assert 0 < im < 2 ** 31

    def fl(x):  # floor(x / s): high word of the signed 64-bit product, >> 20
        return ((x * im) >> 32) >> 20
    deg = (h0 * 360) >> 32
    jb = IDX[deg] - 1  # -1: cut 251 of the turn before
    e64 = h0 + int(float(n) * s) + MA + 4  # past the last ray and its margin
    je = IDX[((e64 % U) * 360 >> 32) + 1] + 252 * (e64 >> 32)
    march, near = [], []
    for ju in range(jb, je):  # the camera's (camera, cut) pairs, packed over the lanes
        j = ju % 252
        cut, cutn = CUT[j], CUT[(j + 1) % 252]
        # every cut lies ahead of h0 by less than the int32 half turn or a little behind it
        # (cuts of h0's own degree): the kernel's signed offsets never wrap (fov < 170)
        ahead = (cutn - h0) % U
        assert ahead < 2 ** 31 - 2 * MA or ahead > U - 6 * UPD
        rel = ((cut - h0 + 2 ** 31) % U) - 2 ** 31
        reln = ((cutn - h0 + 2 ** 31) % U) - 2 ** 31
        mj = MA if cut % (U // 4) == 0 else MT
        mn = MA if cutn % (U // 4) == 0 else MT
        A = fl(rel + mj) + 1
        B = -fl(mj - rel)
        Bn = -fl(mn - reln)
        # the products stay within a signed 64-bit word and agree with the exact quotients
        # to far less than a margin (1.4 units at s = 0.5 degrees)
        assert abs((rel + mj) - (A - 1) * s) <= s + 2 and abs(B * s - (rel - mj)) <= s + 2
        a0 = max(A, 0)
        if a0 <= n and a0 < Bn:
            march.append(j)
        if B < A and 0 <= B <= n:
            near.append(B)
    # the pairs past je hold nothing: the next cut's margin starts past the last ray
    j = je % 252
    rel = ((CUT[j] - h0 + 2 ** 31) % U) - 2 ** 31
    assert -fl((MA if CUT[j] % (U // 4) == 0 else MT) - rel) > n
    return march, near


def _ray(walls, row, col, heading, fov, i, vis):
    """one ray of Camera.get_vision_cone_tiles (security.py:69-99)"""
    R, C = walls.shape
    n = max(int(fov * 2), 30)
    a = math.radians(heading - fov / 2.0 + (fov * i / n))
    dx, dy = math.cos(a), -math.sin(a)
    for k in range(1, 13):
        fx, fy = col + dx * (k * 0.5), row + dy * (k * 0.5)
        c, r = int(round(fx)), int(round(fy))
        if not (0 <= r < R and 0 <= c < C) or walls[r, c]:
            return
        if (r, c) != (row, col):
            vis[r, c] = True


def _march(walls, row, col, dxs, dys, vis):
    R, C = walls.shape
    for k in range(1, 13):
        c, r = col + int(np.rint(k * dxs)), row + int(np.rint(k * dys))
        if not (0 <= r < R and 0 <= c < C) or walls[r, c]:
            return
        if (r, c) != (row, col):
            vis[r, c] = True


def _cone(walls, row, col, heading, fov):
    vis = np.zeros(walls.shape, bool)
    march, near = fan_lanes(heading, fov)
    for j in march:
        _march(walls, row, col, DIRS[j][0], DIRS[j][1], vis)
    for i in near:
        _ray(walls, row, col, heading, fov, i, vis)
    return vis, len(march), len(near)


def _check(walls, row, col, heading, fov):
    got, nm, nn = _cone(walls, row, col, heading, fov)
    want = po.cone(0, walls, row, col, fov, heading, 6)
    assert np.array_equal(got, want), (row, col, heading, fov)
    return nm, nn


def test_partition_matches_oracle_random_cameras():
    rng = np.random.default_rng(11)
    n_march = n_near = 0
    for t in range(1500):
        R = C = 20 if t % 3 else 32
        walls = rng.random((R, C)) < rng.uniform(0.0, 0.25)
        row, col = int(rng.integers(0, R)), int(rng.integers(0, C))
        walls[row, col] = False
        fov = float(np.float32(rng.uniform(30, 120)))  # the synthetic mix (heist_amd/layouts.py)
        heading = float(np.float32(rng.uniform(0, 360)))
        for _ in range(int(rng.integers(1, 4))):  # a few ticks of rotation (security.py:49-51)
            nm, nn = _check(walls, row, col, heading, fov)
            n_march += nm
            n_near += nn
            heading = (heading + float(np.float32(rng.uniform(5, 35)))) % 360.0
    assert n_near < 0.002 * n_march, (n_near, n_march)


def test_partition_widest_fans():
    """fovs up to the eligibility bound (< 170 degrees): the signed cut offsets never wrap,
    and the cones still equal the oracle's."""
    rng = np.random.default_rng(13)
    for t in range(120):
        walls = rng.random((20, 20)) < 0.08
        row, col = int(rng.integers(1, 19)), int(rng.integers(1, 19))
        walls[row, col] = False
        fov = float(np.float32(rng.uniform(150, 169.99)))
        heading = float(np.float32(rng.uniform(0, 360)))
        _check(walls, row, col, heading, fov)


def test_partition_axis_and_cut_rays():
    """Rays exactly on an axis (the reference's default camera, whole and half degrees),
    and rays a few units either side of every cut (inside and just outside the margins)."""
    rng = np.random.default_rng(12)
    walls = np.zeros((20, 20), bool)
    walls[rng.random((20, 20)) < 0.12] = True
    walls[10, 10] = False
    for heading in (0.0, 15.0, 30.0, 45.0, 90.0, 180.0, 270.0, 359.5, 0.5):
        for fov in (60.0, 30.0, 90.0, 120.0, 45.5):
            _check(walls, 10, 10, heading, fov)
    n_near = 0
    for j in range(252):
        for d in (-MA - 3, -MA + 3, -MT - 3, -MT + 3, -1, 0, 1, MT - 3, MT + 3, MA - 3, MA + 3):
            ray_deg = ((CUT[j] + d) % U) / UPD
            fov = float(np.float32(rng.uniform(30, 120)))
            n = max(int(fov * 2), 30)
            i = int(rng.integers(0, n + 1))
            heading = ray_deg + fov / 2.0 - (fov * i / n)  # ray i lands (within rounding) on ray_deg
            heading = heading % 360.0
            row, col = int(rng.integers(2, 18)), int(rng.integers(2, 18))
            w = walls.copy()
            w[row, col] = False
            n_near += _check(w, row, col, heading, fov)[1]
    assert n_near > 0  # the margins were exercised

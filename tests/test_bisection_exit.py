"""The device's Cubic::t_at_y (wg_geom.hip) stops its 40-step bisection once
the midpoint rounds to an end point and returns that midpoint; the reference
(commit_graph.rs:635-654, oracle/wg_oracle.c) always runs 40 steps.  Both must
give the same f32 bits for every input, including NaN / inf control points,
targets next to the end points and sub-ulp intervals.  Vectorised float32
numpy restatement of both loops (per-operation f32 rounding, no FMA)."""
import numpy as np

F = np.float32


def y_at(p, t):
    s = F(1) - t
    return s * s * s * p[0] + F(3) * s * s * t * p[1] + F(3) * s * t * t * p[2] + t * t * t * p[3]


def t_at_y(p, target, early):
    n = target.shape[0]
    out = np.full(n, np.nan, F)
    done = np.zeros(n, bool)
    lo0 = target <= p[0]
    hi1 = ~lo0 & (target >= p[3])
    out[lo0], out[hi1] = F(0), F(1)
    done |= lo0 | hi1
    lo, hi = np.zeros(n, F), np.ones(n, F)
    for _ in range(40):
        mid = (lo + hi) * F(0.5)
        if early:
            stop = ~done & ((mid == lo) | (mid == hi))
            out[stop] = mid[stop]
            done |= stop
        with np.errstate(invalid="ignore", over="ignore"):
            y = y_at(p, mid)
        go = ~done
        lt = go & (y < target)
        lo = np.where(lt, mid, lo)
        hi = np.where(go & ~lt, mid, hi)
    rest = ~done
    out[rest] = ((lo + hi) * F(0.5))[rest]
    return out


def test_early_exit_is_bit_identical():
    rng = np.random.default_rng(7)
    n = 200_000
    y0 = rng.uniform(-1e6, 1e6, n).astype(F)
    dy = rng.choice([rng.uniform(0, 4000, n), rng.uniform(0, 1e-3, n), 10.0 ** rng.uniform(-30, 30, n)]).astype(F)
    p = [y0, (y0 + dy * F(0.4)).astype(F), (y0 + dy - dy * F(0.4)).astype(F), (y0 + dy).astype(F)]
    # targets: uniform inside, next to both end points, outside, NaN
    tgt = (y0 + dy * rng.uniform(-0.1, 1.1, n).astype(F)).astype(F)
    k = n // 8
    tgt[:k] = np.nextafter(p[0][:k], np.inf, dtype=F)
    tgt[k:2 * k] = np.nextafter(p[3][k:2 * k], -np.inf, dtype=F)
    tgt[2 * k:2 * k + 100] = np.nan
    # non-finite and reversed control points
    p[1][3 * k:3 * k + 100] = np.inf
    p[2][3 * k + 100:3 * k + 200] = -np.inf
    p[1][3 * k + 200:3 * k + 300], p[2][3 * k + 200:3 * k + 300] = p[2][3 * k + 200:3 * k + 300], p[1][3 * k + 200:3 * k + 300]
    with np.errstate(invalid="ignore", over="ignore"):
        a = t_at_y(p, tgt, early=False)
        b = t_at_y(p, tgt, early=True)
    assert a.view(np.uint32).tobytes() == b.view(np.uint32).tobytes()

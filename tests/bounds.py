"""The one fp32 tolerance the multi-rank tests use: a sum of
`world` addends in any order is within (world-1)·u·Σ|x| of the exact sum
(u = 2^-24), the / world adds one rounding; two such results (each in its own
order) differ by at most twice that. An SGD / SMA update on top adds the
roundings of its own few operations (u per operation and operand magnitude).
Nothing here is an ad-hoc atol."""

U32 = 2.0 ** -24


def avg_bound(addends, world):
    """Bound on |a - b| for two fp32 averages of the same `world` addends
    summed in different orders: 2·((world-1)·u·Σ|x| / world + u·|avg|)."""
    ab = sum(a.double().abs() for a in addends)
    avg = sum(a.double() for a in addends) / world
    return 2 * ((world - 1) * U32 * ab / world + U32 * avg.abs())


def sgd_bound(avg_b, lr, p, g):
    """p' = p - lr·g with g known to avg_b: lr·avg_b plus the update's own
    roundings on either side (the product and the difference, or one FMA)."""
    return lr * avg_b + 2 * U32 * (p.double().abs() + lr * g.double().abs())


def sma_bound(avg_b, alpha, v, avg):
    """v' = (1-a)·v + a·avg with avg known to avg_b: a·avg_b plus two products
    and a sum rounded on either side."""
    return alpha * avg_b + 4 * U32 * ((1 - alpha) * v.double().abs() + alpha * avg.double().abs())


def assert_within(got, want, bound, what=""):
    d = (got.double() - want.double()).abs()
    bad = d > bound.to(d.device) * (1 + 1e-9)
    assert not bool(bad.any()), "%s: %d elements beyond the bound (max excess %g)" % (
        what, int(bad.sum()), float((d - bound.to(d.device)).max()))

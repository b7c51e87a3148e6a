"""The GPU field arithmetic never overflows: an interval restatement of every
product, carry chain and group formula the kernels use
(tests/bounds_model.py), checked against the machine types (int32
multiply operands and limb sums, int64 column accumulators) for inputs
anywhere in their documented ranges, and iterated over the dsm loop until
the intervals stop growing."""
import pytest

import bounds_model as bm


def _within(f, lo_mult, hi_mult):
    """every limb of f within [lo_mult, hi_mult] x (2^25 even, 2^24 odd)"""
    for k, (lo, hi) in enumerate(f):
        unit = 1 << (bm.W[k] - 1)
        assert lo >= lo_mult * unit and hi <= hi_mult * unit, (k, lo, hi, unit)


def test_centered_products_are_tight():
    x = [(-int(3.3 * (1 << (w - 1))), int(3.3 * (1 << (w - 1)))) for w in bm.W]
    _within(bm.fe_mul(x, x), -1.01, 1.01)
    _within(bm.fe_sqs(x), -1.01, 1.01)
    _within(bm.fe_sqs(x, 2), -1.01, 1.01)


def test_unsigned_products_stay_in_two_units():
    x = [(-int(3.3 * (1 << (w - 1))), int(3.3 * (1 << (w - 1)))) for w in bm.W]
    for f in (bm.fe_mul_u(x, x), bm.fe_sqs_u(x), bm.fe_sqs_u(x, 2)):
        _within(f, -0.001, 2.001)


def test_unsigned_chain_is_a_fixed_point():
    u = bm.fe_sqs_u(bm.frombytes())
    assert bm.fe_sqs_u(u) == bm.fe_sqs_u(bm.fe_sqs_u(u))
    assert bm.fe_mul_u(u, u) == bm.fe_mul_u(bm.fe_mul_u(u, u), u)


def test_19_side_limit_is_real():
    """the model rejects what the device could not compute: a 4x operand on
    the 19-side overflows the 32-bit multiply operand"""
    x4 = [(0, 4 << (w - 1)) for w in bm.W]
    with pytest.raises(bm.Overflow):
        bm.fe_mul_u(bm.frombytes(), x4)


def test_exponentiation_chain():
    for z in (bm.centered_tight(), bm.frombytes(), bm.fe_mul(bm.centered_tight(), bm.centered_tight())):
        _within(bm.fe_pow22523(z), -0.001, 2.001)


def test_group_operations_standalone():
    u = bm.fe_sqs_u(bm.frombytes())   # an unsigned output
    p2 = {"X": u, "Y": u, "Z": u}
    r = bm.p2_dbl(p2)
    for k in "XYZT":
        _within(r[k], -3.04, 3.04)
    q = bm.table_entries(True)
    for k in ("YplusX", "YminusX", "Z2"):
        _within(q[k], -3.04, 3.04)


@pytest.mark.parametrize("loop", [bm.dsm_half_loop, bm.dsm_full_loop])
def test_dsm_loop_fixed_point(loop):
    Q, iters = loop()
    assert iters < 6, "intervals did not converge"
    for k in "XYZ":
        _within(Q[k], -0.001, 2.001)


def test_formula_choices_are_needed():
    """the alternatives the kernels avoid do overflow: (X+Y)^2 of unsigned
    coordinates, and 2dT from a -2dT table as a 19-side"""
    u = bm.fe_sqs_u(bm.frombytes())
    with pytest.raises(bm.Overflow):
        bm.fe_sqs_u(bm.fe_add(u, u))
    r = bm.ge_add({"X": u, "Y": u, "Z": u, "T": u}, bm.table_entries(True), True)
    with pytest.raises(bm.Overflow):
        bm.fe_mul19_u(r["X"], r["T"], bm.fe_19(r["T"]))

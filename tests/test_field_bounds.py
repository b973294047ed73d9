"""Worst-case column bounds of the radix-2^25.5 field multiply (narwhal_amd/csrc/nw_field.hpp).

fe_mul / fe_sq accumulate each of the 10 output columns in one 64-bit register and fold the
previous column's carry in as the initial accumulator, so every column sum plus its
carry-in must stay below 2^64 for every operand pair the point formulas
(narwhal_amd/csrc/nw_point.hpp) feed it. The limb bounds are the ones nw_field.hpp states:
T (carried output), L = T + T, P15 = T + L, S(x) = x + 4p (fe_sub_nc, no carry).
"""
import math

P4 = [4 * (2**26 - 19)] + [4 * (2**26 - 1) if i % 2 == 0 else 4 * (2**25 - 1) for i in range(1, 10)]
T = [2**26 if i % 2 == 0 else 2**25 for i in range(10)]
T[1] += 2**17          # fe_join / fold_top: limb 1 receives the wrapped carry (< 2^17)
T[6] += 2**13          # fe_join: limb 6 receives the column-4 carry (< 2^13)
L = [2 * x for x in T]
P15 = [a + b for a, b in zip(T, L)]
S_T = [a + b for a, b in zip(T, P4)]      # fe_sub_nc(T, T)
S_L = [a + b for a, b in zip(L, P4)]      # fe_sub_nc(L, T)


def colmax(F, G):
    cols = [0] * 10
    for i in range(10):
        for j in range(10):
            m = F[i] * G[j] * (2 if (i % 2 and j % 2) else 1)
            k = i + j
            if k >= 10:
                m *= 19
                k -= 10
            cols[k] += m
    return max(cols)


def carry_in(col):
    return col >> 25


# every (first, second) operand-bound pair the formulas produce (nw_point.hpp); the first
# operand's odd limbs are doubled and the second's limbs are scaled by 19 in 32 bits
MUL_PAIRS = {
    "a*YmX, c = neg(2dT)*T, X3 = e*f": (S_T, T),
    "T3 = e*h; sub_cached X3 = e*f, Y3 = g*h, Z3 = g*f": (S_T, L),
    "Z3 = f*g": (T, P15),
    "Y3 = g*h": (P15, L),
    "dbl X3 = E*F": (S_L, P15),
    "dbl T3 = E*H": (S_L, L),
    "dbl Z3 = F*G": (P15, T),
    "generic": (T, T),
}
SQ_INPUTS = {"X, Y, Z": T, "X+Y": L}


def test_mul_columns_and_32bit_scalings():
    for name, (F, G) in MUL_PAIRS.items():
        c = colmax(F, G)
        assert c + carry_in(c) < 2**64, (name, math.log2(c))
        assert max(G) * 19 < 2**32, name          # g_i * 19
        assert max(F[1::2]) * 2 < 2**32, name     # f_odd * 2


def test_sq_columns_and_32bit_scalings():
    for name, F in SQ_INPUTS.items():
        # fe_sq's columns are the same sums as fe_mul(f, f)
        c = colmax(F, F)
        assert c + carry_in(c) < 2**64, name
        assert max(F[5::2]) * 38 < 2**32, name    # f5, f7, f9 * 38
        assert max(F[6::2]) * 19 < 2**32, name    # f6, f8 * 19
        assert max(F) * 2 < 2**32, name


def test_uncarried_operand_needs_first_slot():
    # why fe_sub_nc results may not be fe_mul's second operand
    assert max(S_T) * 19 >= 2**32

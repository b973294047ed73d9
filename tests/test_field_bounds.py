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
# fe_join5 (five two-column chains): chain c's final carry (< 2^64 >> 25 = 2^39) enters limb
# 2c + 2 (x 19 into limb 0), which is re-split once, so limb 2c + 3 receives < 2^13 + 1
# (limb 1: < 2^17.25 + 1); the old two-chain fe_join fed limbs 1 and 6 the same way.
T[1] += (19 * 2**39 + 2**26) >> 26
for i in (3, 5, 7, 9):
    T[i] += (2**39 + 2**26) >> 26
T[6] += (2**39 + 2**26) >> 26   # fe_join (NW_MAC_CHAINS=2)
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
    "dbl Z3 = G*F (shared second operand F)": (T, P15),
    "add Z3 = g*f (shared second operand f)": (L, T),
    "generic": (T, T),
    # ge_add_any_negc (NW_ADD_NEGC): f = d + c' (L cached, P15 affine d = 2Z) second,
    # g = d - c' uncarried (S_T cached, S_L affine) first
    "negc X3 = e*f (cached)": (S_T, L),
    "negc Z3 = g*f, Y3 = g*h (cached)": (S_T, L),
    "negc X3 = e*f (affine)": (S_T, P15),
    "negc Z3 = g*f (affine)": (S_L, P15),
    "negc Y3 = g*h (affine)": (S_L, L),
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


# Limb-parallel arithmetic (narwhal_amd/csrc/nw_lp.hpp, the Horner of k_pip_final): products
# are carried in two parallel passes, so limb 0 may hold up to 2^26 + 2^18.3 (19 x the
# second-pass carry from limb 9), limb 1 up to 2^25 + 2^17.3 and the rest up to
# 2^26 / 2^25 + 2^14; one-pass carried differences stay inside that.
T_LP = [2**26 + 2**18.3 if i == 0 else 2**25 + 2**17.3 if i == 1 else
        (2**26 if i % 2 == 0 else 2**25) + 2**14 for i in range(10)]
T_LP = [int(x) + 1 for x in T_LP]


def test_limb_parallel_bounds():
    L_ = [2 * x for x in T_LP]
    P15_ = [a + b for a, b in zip(T_LP, L_)]
    S_T_ = [a + b for a, b in zip(T_LP, P4)]
    S_L_ = [a + b for a, b in zip(L_, P4)]
    pairs = [(S_T_, T_LP), (S_T_, L_), (T_LP, P15_), (P15_, L_), (S_L_, P15_), (S_L_, L_),
             (P15_, T_LP), (T_LP, T_LP), (T_LP, T_LP), (L_, L_)]
    for F, G in pairs:
        c = colmax(F, G)
        assert c < 2**64
        assert max(G) * 19 < 2**32 and max(F[1::2]) * 2 < 2**32   # NW_LP_XLANE=0
        assert max(G[0::2]) * 19 < 2**32 and max(G[1::2]) * 38 < 2**32   # NW_LP_XLANE=1: x2 on g
    # first pass: carries < 2^39 (x19 < 2^43.3 into limb 0); second: < 2^18.3 into limb 0
    assert (2**64 >> 25) * 19 < 2**44
    assert 19 * (((2**25 + 2**39) >> 25) + 1) < 2**18.3
    assert ((2**26 + 19 * 2**39) >> 26) < 2**17.3
    # one-pass lp_sub: a + 4p - b < 2^29, carry < 2^4, x19 into limb 0 < 2^9
    assert max(a + b for a, b in zip(P15_, P4)) < 2**29
    assert 19 * (2**29 >> 25) < 2**18.3

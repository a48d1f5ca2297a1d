"""Crafted scalars and records for the per-key comb tables (verify.h
lltab_build / q_llcomb: the signed Lim-Lee comb of one-lane-per-record
batches), shared by the host-harness tests and the GPU tests.

A record built for a chosen u2 (R = u1 G + u2 Q, r = x(R) mod n, s = r / u2,
e = u1 s) verifies by construction; its flipped-digest twin fails (R_MATH).
The scalars sit at the signed comb's edges: odd and even u2 (k = u2 or u2 + n),
columns whose lower teeth are all clear or all set, a top tooth of zeros
(negated entries in every column), single digits, the largest k, and u2 whose
Horner hits A == V_j (the doubling branch) -- found by running the comb's
recurrence on every sign pattern of column 0 (the infinity branch A == -V_j
cannot occur for these shapes: tests/comb_cases.py::horner_events).
"""
from __future__ import annotations

import itertools
import random

from oracle import ecdsa_ref as O


def horner_events(u2: int, n: int, t: int, s: int):
    """The signed comb's Horner on the scalar u2 (verify.h q_llcomb), as
    integers mod n: [(event, column)] for the degenerate steps."""
    k = u2 if u2 & 1 else u2 + n
    c = (k >> 1) | (1 << (t * s - 1))
    V = [sum((2 * ((c >> (s * i + j)) & 1) - 1) << (s * i) for i in range(t)) for j in range(s)]
    assert sum(v << j for j, v in enumerate(V)) == k
    ev, a, inf = [], V[s - 1], False
    for j in range(s - 2, -1, -1):
        a *= 2
        if inf:
            a, inf = V[j], False
            ev.append(("from_inf", j))
            continue
        if (a - V[j]) % n == 0:
            ev.append(("dbl", j))
        elif (a + V[j]) % n == 0:
            ev.append(("inf", j))
            a, inf = 0, True
            continue
        a += V[j]
    assert inf or (a - k) % n == 0
    return ev


def signed_comb_u2(n: int, t: int, s: int, seed: int = 5) -> list[int]:
    """u2 at the edges of the t x s signed comb for group order n."""
    ts = t * s
    out = [1, 2, 3, n - 1, n - 2, n // 2, n // 2 + 1, 2**255, (2**256) % n, 2**(s * (t - 1)),
           2**(s * (t - 1)) + 1, 2**s, 2**s + 1, 2**(s - 1)]

    def from_c(x):  # c = 2^(ts-1) + x  ->  k = 2 x + 1 -> u2
        k = 2 * x + 1
        return (k if k < n else k - n) if k < 2 * n else None

    lower_all = 2**(s * (t - 1)) - 1
    patterns = [0, lower_all, lower_all ^ ((2**s - 1) << (s * (t - 2))),  # top tooth 0
                sum(1 << (s * i) for i in range(t - 1)),               # one column full
                sum(((2**s - 1) if i % 2 else 0) << (s * i) for i in range(t - 1)),
                sum((0x5555555555555555 & ((1 << s) - 1)) << (s * i) for i in range(t - 1)),
                n - 1 - (2**(ts - 1) % n) if ts - 1 < 256 else (n - 1) // 2]
    for x in patterns:
        u2 = from_c(x)
        if u2:
            out.append(u2)
    # the doubling branch: k == 2 V_0 (mod n) for a sign pattern of column 0
    for pat in itertools.product((-1, 1), repeat=t):
        v0 = sum(d << (s * i) for i, d in enumerate(pat))
        u2 = (2 * v0) % n
        if u2 and any(e[0] == "dbl" for e in horner_events(u2, n, t, s)):
            out.append(u2)
    rng = random.Random(seed)
    out += [rng.randrange(1, n) for _ in range(4)]
    seen, res = set(), []
    for u in out:
        u %= n
        if u and u not in seen:
            seen.add(u)
            res.append(u)
    return res


def unsigned_comb_u2(t: int, s: int) -> list[int]:
    """Round 3's crafted scalars for the unsigned t x s comb (single teeth,
    empty / full top columns): still a spread of column patterns."""
    top = 256 - s * (t - 1)
    return [2**(s - 1), 2**s, 2**(2 * s), 2**(s * (t - 1)), 2**255,
            2**(s * (t - 1)) + 2**(s * (t - 1) - 1), 2**s - 1,
            sum(2**(s * k) for k in range(t)), sum(2**(s * k + s - 1) for k in range(t - 1)),
            sum(2**(s * k + s - 1) for k in range(t - 1)) + 2**255,
            (2**s - 1) << (256 - top - s), sum((2**s - 1) << (s * k) for k in range(t - 1))]


def g_comb_u1(n: int, gw: int) -> list[int]:
    """u1 at the edges of the kGW-bit signed-window G comb (verify.h g_comb):
    zero windows (digit 0 keeps B), the most negative digit -2^(kGW-1) (the
    table's last entry), all-ones windows (carries through the recoding),
    single windows, n - 1."""
    nw = -(-257 // gw)
    half, full = 2**(gw - 1), 2**gw - 1
    out = [1, 2, 3, n - 1, n - 2, n // 2, 2**gw, 2**(gw * (nw - 1)), 2**255,
           sum(half << (gw * w) for w in range(nw - 1)) % n,          # every digit -2^(kGW-1)
           sum(full << (gw * w) for w in range(nw - 1)) % n,          # carries all the way
           sum((half if w % 2 else 0) << (gw * w) for w in range(nw - 1)) % n,
           sum(1 << (gw * w) for w in range(0, nw - 1, 3)) % n]       # zero windows between
    return [u % n for u in out if u % n]


def records_for_u2(curve, u2s, seed: int = 77, d: int | None = None, low_s: bool = False,
                   u1s=None):
    """One key; per u2 a valid signature and its flipped-digest twin:
    [(qx, qy, der_sig, digest)], the first verifying, the twin R_MATH. With
    low_s, u1 is redrawn until s <= n / 2, so the signature passes Fabric's
    low-S rule AND the verifier still computes exactly this u2."""
    c = curve
    n = c.n
    rng = random.Random(seed)
    d = d or rng.randrange(1, n)
    qx, qy = O.scalar_mult(c, d, (c.gx, c.gy))
    recs = []
    for k, u2 in enumerate(u2s):
        u2Q = O.scalar_mult(c, u2 % n, (qx, qy))
        for tries in range(64):
            if u1s:  # chosen u1: for low-S, redraw u2 instead
                u1 = u1s[k % len(u1s)]
                if tries:
                    u2 = rng.randrange(1, n)
                    u2Q = O.scalar_mult(c, u2, (qx, qy))
            else:
                u1 = rng.randrange(1, n)
            R = O.point_add(c, O.scalar_mult(c, u1, (c.gx, c.gy)), u2Q)
            if R is None or R[0] % n == 0:
                continue
            r = R[0] % n
            s = r * pow(u2, -1, n) % n
            if not low_s or s <= n // 2:
                break
        else:
            continue
        e = u1 * s % n
        for dg in (e.to_bytes(32, "big"), (e ^ 1).to_bytes(32, "big")):
            recs.append((qx, qy, O.marshal_ecdsa_signature(r, s), dg))
    return recs


# ---- u1 G folded into the key comb's Horner (round 5, verify.h q_llcomb_g) ----
def comb_columns(u: int, n: int, t: int, s: int) -> list[int]:
    """The signed comb's column values V_j (u = sum 2^j V_j mod n)."""
    k = u if u & 1 else u + n
    c = (k >> 1) | (1 << (t * s - 1))
    return [sum((2 * ((c >> (s * i + j)) & 1) - 1) << (s * i) for i in range(t)) for j in range(s)]


def fold_events(u1: int, u2: int, d: int, n: int, t: int, s: int, kgf: int = 2):
    """The folded Horner (q_llcomb_g) on u1 G + u2 Q with Q = d G, as integers
    mod n (multiples of G), in the kernel's order: load the top column of u2;
    per column j = s-2 .. 0 the composite A = 2 A + V_j Q computed as
    (A + T) + A (ll_dbladd, kind "Q": A == T -> "dbl", A == -T -> "neg",
    2 A + T == 0 -> "inf"), then at the lowest column j of each group of kgf
    u1 columns (j = 1, 1 + kgf, ...) the group's point sum_c 2^c W_(j+c), and
    at j = 0 the u1 column 0 (a mixed addition, kind "G": A == T -> "dbl",
    A == -T -> "inf"). Returns ([(event, column, kind)], total is infinity)."""
    V, W = comb_columns(u2, n, t, s), comb_columns(u1, n, t, s)
    ev, a, inf = [], V[s - 1] * d % n, False
    for j in range(s - 2, -1, -1):
        T = V[j] * d % n
        if inf:
            a, inf = T, False
            ev.append(("from_inf", j, "Q"))
        elif (a - T) % n == 0:
            ev.append(("dbl", j, "Q"))
            a = 3 * T % n
        elif (a + T) % n == 0:
            ev.append(("neg", j, "Q"))
            a = -T % n
        elif (2 * a + T) % n == 0:
            ev.append(("inf", j, "Q"))
            a, inf = 0, True
        else:
            a = (2 * a + T) % n
        adds = []
        if j >= 1 and (j - 1) % kgf == 0:
            adds.append(("G", sum(W[j + c] << c for c in range(kgf)) % n))
        if j == 0:
            adds.append(("G", W[0] % n))
        for kind, T in adds:
            if inf:
                a, inf = T, False
                ev.append(("from_inf", j, kind))
            elif (a - T) % n == 0:
                ev.append(("dbl", j, kind))
                a = 2 * T % n
            elif (a + T) % n == 0:
                ev.append(("inf", j, kind))
                a, inf = 0, True
            else:
                a = (a + T) % n
    assert (inf and (u1 + u2 * d) % n == 0) or (not inf and a == (u1 + u2 * d) % n)
    return ev, inf


def fold_crafted(curve, t: int, s: int, seed: int = 17, tries: int = 20000,
                 low_s: bool = False, kgf: int = 2):
    """(u1, u2, d) triples whose folded Horner takes each degenerate branch
    reachable by construction -- the last columns, where the remaining sum can
    be solved for: u1's column-0 entry doubling / cancelling the sum (the
    single-column table), u2's column-0 composite 2 A + T meeting A == T,
    A == -T and 2 A + T == 0, the column-1 pair entry doubling / cancelling
    the sum, and u2's column-1 composite cancelling it (the pair then taken
    from infinity). u1 is drawn, u2 is
    solved from the wanted total u1 + u2 d, and kept when its own column
    pattern matches the one the total assumed (~1/2^t). low_s: a finite
    R = u1 G + u2 Q must give s = x(R) / u2 <= n / 2 (Fabric's rule), else the
    draw is discarded."""
    import random
    n = curve.n
    rng = random.Random(seed)
    want = {("dbl", 0, "G"), ("inf", 0, "G"), ("dbl", 0, "Q"), ("neg", 0, "Q"),
            ("inf", 0, "Q"), ("dbl", 1, "G"), ("inf", 1, "G"), ("inf", 1, "Q")}
    found, out = set(), []
    for _ in range(tries):
        if found == want:
            break
        d = rng.randrange(1, n)
        u1 = rng.randrange(1, n)
        W = comb_columns(u1, n, t, s)
        p = [rng.choice((-1, 1)) for _ in range(t)]
        v0 = sum(x << (s * i) for i, x in enumerate(p))
        pair1 = sum(W[1 + c] << c for c in range(kgf))  # the G group added at column 1
        targets = {  # event -> the total u1 + u2 d it needs (v0 = u2's assumed column 0)
            ("dbl", 0, "G"): 2 * W[0],
            ("inf", 0, "G"): 0,
            ("dbl", 0, "Q"): 3 * v0 * d + W[0],
            ("neg", 0, "Q"): -v0 * d + W[0],
            ("inf", 0, "Q"): W[0],
            ("dbl", 1, "G"): 4 * pair1 + v0 * d + W[0],
            ("inf", 1, "G"): v0 * d + W[0],
            ("inf", 1, "Q"): 2 * pair1 + v0 * d + W[0],
        }
        for key, total in targets.items():
            if key in found:
                continue
            u2 = (total - u1) * pow(d, -1, n) % n
            if not u2:
                continue
            ev, inf = fold_events(u1, u2, d, n, t, s, kgf)
            if key not in [e for e in ev if e[0] != "from_inf"][:1]:
                continue
            if low_s and not inf:
                q = O.scalar_mult(curve, d, (curve.gx, curve.gy))
                r = O.double_scalar(curve, u1, u2, q)[0] % n
                if r == 0 or r * pow(u2, -1, n) % n > n // 2:
                    continue
            found.add(key)
            out.append((u1, u2, d, key, inf))
    return out


def records_for_fold(curve, triples, seed: int = 23, low_s: bool = True):
    """Per (u1, u2, d): records whose verify computes exactly these u1, u2
    with Q = d G -- [(qx, qy, der_sig, digest, expected reason)]. A finite
    R = u1 G + u2 Q gives the valid signature (r = x(R) mod n, s = r / u2,
    e = u1 s) and its flipped-digest twin (R_MATH); R at infinity gives one
    record with any r (it must fail, R_MATH). With low_s, a high s is
    answered by scaling: (u1, u2) -> (c u1, c u2) changes the events, so such
    triples are dropped instead."""
    import random
    n = curve.n
    rng = random.Random(seed)
    out = []
    for u1, u2, d, _key, inf in triples:
        qx, qy = O.scalar_mult(curve, d, (curve.gx, curve.gy))
        if inf:
            for _ in range(64):
                r = rng.randrange(1, n)
                s_ = r * pow(u2, -1, n) % n
                if not low_s or s_ <= n // 2:
                    break
            else:
                continue
            e = u1 * s_ % n
            out.append((qx, qy, O.marshal_ecdsa_signature(r, s_), e.to_bytes(32, "big"), 9))
            continue
        R = O.double_scalar(curve, u1, u2, (qx, qy))
        r = R[0] % n
        if r == 0:
            continue
        s_ = r * pow(u2, -1, n) % n
        if low_s and s_ > n // 2:
            continue
        e = u1 * s_ % n
        sig = O.marshal_ecdsa_signature(r, s_)
        out.append((qx, qy, sig, e.to_bytes(32, "big"), 0))
        out.append((qx, qy, sig, (e ^ 1).to_bytes(32, "big"), 9))
    return out


# ---- the variable-base ladder with u1 G folded in (round 5, verify.h q_ladder_odd_g) ----
def ladder_digits(u2: int, n: int):
    """Odd signed 5-bit windows of k = u2 (odd) or u2 + n: (top digit, [d_0 .. d_50])."""
    k = u2 if u2 & 1 else u2 + n
    d = [2 * ((k >> (5 * i + 1)) & 31) - 31 for i in range(51)]
    top = 2 * ((k >> 256) & 1) + 1
    assert (top << 255) + sum(x << (5 * i) for i, x in enumerate(d)) == k
    return top, d


def ladder_events(u1: int, u2: int, d: int, n: int, t: int = 7, s: int = 37, kgf: int = 3):
    """q_ladder_odd_g on u1 G + u2 Q (Q = d G) as integers mod n, in the
    kernel's order: A = top digit Q; per window 50 .. 0: 4 doublings, each
    followed by the folded G group whose weight exponent equals the doublings
    still to come (p = 0, 1, 1 + kgf, ..., s - kgf), then the composite
    2 A + d_i Q (kind "Q": "dbl" A == T, "neg" A == -T, "inf" 2 A + T == 0)
    and the G entry at p = 5 i. G additions: kind "G<p>" ("dbl" / "inf").
    Returns ([(event, window, kind)], total is infinity)."""
    top, dig = ladder_digits(u2, n)
    W = comb_columns(u1, n, t, s)

    def gpos(p):
        return p == 0 or (1 <= p <= s - kgf and (p - 1) % kgf == 0)

    def gval(p):
        return W[0] if p == 0 else sum(W[p + c] << c for c in range(kgf))
    ev, a, inf = [], top * d % n, False

    def gadd(win, p):
        nonlocal a, inf
        T = gval(p) % n
        if inf:
            a, inf = T, False
            ev.append(("from_inf", win, f"G{p}"))
        elif (a - T) % n == 0:
            ev.append(("dbl", win, f"G{p}"))
            a = 2 * T % n
        elif (a + T) % n == 0:
            ev.append(("inf", win, f"G{p}"))
            a, inf = 0, True
        else:
            a = (a + T) % n
    for win in range(50, -1, -1):
        for dd in range(1, 5):
            if not inf:
                a = 2 * a % n
            if gpos(5 * win + 5 - dd):
                gadd(win, 5 * win + 5 - dd)
        T = dig[win] * d % n
        if inf:
            a, inf = T, False
            ev.append(("from_inf", win, "Q"))
        elif (a - T) % n == 0:
            ev.append(("dbl", win, "Q"))
            a = 3 * T % n
        elif (a + T) % n == 0:
            ev.append(("neg", win, "Q"))
        elif (2 * a + T) % n == 0:
            ev.append(("inf", win, "Q"))
            a, inf = 0, True
        else:
            a = (2 * a + T) % n
        if gpos(5 * win):
            gadd(win, 5 * win)
    assert (inf and (u1 + u2 * d) % n == 0) or (not inf and a == (u1 + u2 * d) % n)
    return ev, inf


def ladder_crafted(curve, seed: int = 19, tries: int = 20000, low_s: bool = False,
                   kgf: int = 3, t: int = 7, s: int = 37):
    """(u1, u2, d) triples whose folded ladder takes each degenerate branch
    reachable by construction in the last window: the column-0 G entry
    doubling / cancelling the sum, the composite of digit d_0 meeting A == T,
    A == -T and 2 A + T == 0, the G groups at weight 2^1 and 2^(1 + kgf)
    doubling / cancelling the partial sum. u1 is drawn, u2 solved from the
    total u1 + u2 d each event needs, kept when u2's own d_0 is the digit
    assumed (~1/32). Every triple has its own d (one event per draw), so a
    key carries two records (the valid signature and its twin) and stays
    below kMinUses: no per-batch key table, every record on the ladder."""
    import random
    n = curve.n
    rng = random.Random(seed)
    g4 = 1 + kgf
    want = {("dbl", 0, "G0"), ("inf", 0, "G0"), ("dbl", 0, "Q"), ("neg", 0, "Q"),
            ("inf", 0, "Q"), ("dbl", 0, "G1"), ("inf", 0, "G1"), ("dbl", 0, f"G{g4}"),
            ("inf", 0, f"G{g4}")}
    found, out = set(), []
    for _ in range(tries):
        if found == want:
            break
        d = rng.randrange(1, n)
        u1 = rng.randrange(1, n)
        W = comb_columns(u1, n, t, s)
        G1 = sum(W[1 + c] << c for c in range(kgf))
        G4 = sum(W[g4 + c] << c for c in range(kgf))
        d0 = rng.choice([x for x in range(-31, 32, 2)])
        sh = 2 ** (g4 - 1)  # doublings between the G4 and G1 additions, times 2
        targets = {
            ("dbl", 0, "G0"): 2 * W[0],
            ("inf", 0, "G0"): 0,
            ("dbl", 0, "Q"): 3 * d0 * d + W[0],
            ("neg", 0, "Q"): -d0 * d + W[0],
            ("inf", 0, "Q"): W[0],
            ("dbl", 0, "G1"): 4 * G1 + d0 * d + W[0],
            ("inf", 0, "G1"): d0 * d + W[0],
            ("dbl", 0, f"G{g4}"): 2 * (2 * sh * G4 + G1) + d0 * d + W[0],
            ("inf", 0, f"G{g4}"): 2 * G1 + d0 * d + W[0],
        }
        for key, total in targets.items():
            if key in found:
                continue
            u2 = (total - u1) * pow(d, -1, n) % n
            if not u2 or ladder_digits(u2, n)[1][0] != d0:
                continue
            ev, inf = ladder_events(u1, u2, d, n, t, s, kgf)
            if key not in [e for e in ev if e[0] != "from_inf"][:1]:
                continue
            if low_s and not inf:
                q = O.scalar_mult(curve, d, (curve.gx, curve.gy))
                r = O.double_scalar(curve, u1, u2, q)[0] % n
                if r == 0 or r * pow(u2, -1, n) % n > n // 2:
                    continue
            found.add(key)
            out.append((u1, u2, d, key, inf))
            break  # one event per key: a key stays below the table threshold
    return out


def distinct_key_classes(curve, seed: int = 61, reps: int = 4):
    """The golden file's group-equation classes rebuilt on a fresh key per
    record (tests/golden/gen_golden.py builds them on shared keys): x(R) in
    [n, p) accepted through x mod n == r (u1 = 0 as in the golden record, and
    a random u1), u1 G + u2 Q = infinity, and u1 G == u2 Q (the final addition
    doubles). Q is solved from the wanted R: Q = u2^-1 (R - u1 G).
    [(qx, qy, der_sig, digest, expected reason, tag)]; reason 0 verifies,
    9 = R_MATH (the (false, nil) of verifyNISTEC)."""
    c = curve
    n, p = c.n, c.p
    rng = random.Random(seed)
    G = (c.gx, c.gy)

    def neg(P):
        return (P[0], (-P[1]) % p)

    def wrap_point():
        while True:
            x = n + rng.randrange(p - n)
            rhs = (x * x * x + c.a * x + c.b) % p
            y = pow(rhs, (p + 1) // 4, p)
            if y * y % p == rhs:
                return x, y

    def low_s_u2(r):  # u2 with s = r / u2 <= n / 2
        while True:
            u2 = rng.randrange(1, n)
            s = r * pow(u2, -1, n) % n
            if s <= n // 2:
                return u2, s

    out = []
    for _ in range(reps):
        # x-wrap: R fixed, r = x(R) - n
        for u1_zero in (True, False):
            R = wrap_point()
            r = R[0] - n
            u2, s = low_s_u2(r)
            u1 = 0 if u1_zero else rng.randrange(1, n)
            RmG = R if u1 == 0 else O.point_add(c, R, neg(O.scalar_mult(c, u1, G)))
            Q = O.scalar_mult(c, pow(u2, -1, n), RmG)
            e = u1 * s % n
            sig = O.marshal_ecdsa_signature(r, s)
            out.append((Q[0], Q[1], sig, e.to_bytes(32, "big"), 0, "xwrap_accept"))
            R2 = wrap_point()  # R = R2 again, but r = x(R2) - n + 1: its own key
            r2 = R2[0] - n
            u2, s = low_s_u2(r2 + 1)
            Q2 = O.scalar_mult(c, pow(u2, -1, n), R2)
            out.append((Q2[0], Q2[1], O.marshal_ecdsa_signature(r2 + 1, s), b"\0" * 32, 9,
                        "xwrap_wrong_r"))
        # u1 G + u2 Q = infinity: Q = -(u1 / u2) G
        r = rng.randrange(1, n)
        u2, s = low_s_u2(r)
        u1 = rng.randrange(1, n)
        Q = neg(O.scalar_mult(c, u1 * pow(u2, -1, n) % n, G))
        out.append((Q[0], Q[1], O.marshal_ecdsa_signature(r, s), (u1 * s % n).to_bytes(32, "big"),
                    9, "sum_infinity"))
        # u1 G == u2 Q: Q = (u1 / u2) G, R = 2 u1 G
        for wrong in (False, True):
            u1 = rng.randrange(1, n)
            r = O.scalar_mult(c, 2 * u1 % n, G)[0] % n
            rr = r if not wrong else (r % (n - 1)) + 1  # the verifier still doubles
            u2, s = low_s_u2(rr)
            Q = O.scalar_mult(c, u1 * pow(u2, -1, n) % n, G)
            out.append((Q[0], Q[1], O.marshal_ecdsa_signature(rr, s),
                        (u1 * s % n).to_bytes(32, "big"), 9 if wrong else 0,
                        "u1G_eq_u2Q_wrong_r" if wrong else "u1G_eq_u2Q_accept"))
    return out

#!/usr/bin/env python3
"""numpy model of the register-resident L = 16 384 overlap-save unit
(csrc/fir_fft16r.hpp), zero-phase form: two 256-thread workgroups per CU, each
holding one unit in registers.  It runs the kernel's data flow thread by
thread -- every register index, LDS slot and pair-table slot -- and checks

  * each LDS exchange round: every slot written once, every read gets the
    value the index algebra says, b128 stores conflict-free in their 8-lane
    groups and b128 loads in their 16-lane groups (as scripts/fft32r_model.py);
  * the forward spectrum after stage 3 against numpy's FFT;
  * the outputs against a direct convolution.

The transform: N = 8 192 complex points z[m] = x_seg[2m] + i x_seg[2m+1],
m = 256 n + b (thread b of 256, register n of 32), b = 16 beta + gamma.
  stage 1 (thread b): DFT32 over n -> k1, * W_N^(b k1)
  T1 (workgroup, 2 rounds: registers 0..15, then 16..31): lane (w, s, gamma)
     gathers beta = 0..15 of column P = 4 w + s in round 1 (pair A) and of
     its mirror 32 - P (column 16 for P = 0) in round 2 (pair B)
  stage 2 (both pairs): DFT16 over beta -> kappa, * W_256^(gamma kappa)
  T2 (16-lane groups, 2 rounds: kappa < 8, then kappa >= 8): lane (w, s, q)
     gathers gamma for task R1 (column, kappa < 8) and its mirror task R2
     (32 - column, 15 - kappa)
  stage 3: DFT16 over gamma -> lambda:  Z[k1 + 32 kappa + 512 lambda]
  pair step (R1[i] with R2[15 - i]), then the same stages backwards.
usage: fft16r_model.py [ntaps]
"""
import sys

import numpy as np

N = 8192
L = 2 * N
NT = 256
NW = NT // 64
RG = 1088  # double2 per wave region (T2 rows padded to 17 slots)


# ---- column ownership -------------------------------------------------------
def pair_cols(w, s):
    """(column of pair A, column of pair B) of 16-lane group s of wave w"""
    P = 4 * w + s
    return (0, 16) if P == 0 else (P, 32 - P)


COL_OF = {}  # k1 -> (w, s, pair)
for w in range(NW):
    for s in range(4):
        a, b = pair_cols(w, s)
        COL_OF[a] = (w, s, 0)
        COL_OF[b] = (w, s, 1)
assert sorted(COL_OF) == list(range(32))


# ---- T2 task assignment -----------------------------------------------------
def t2_tasks(w, s, q):
    """(pair, kappa) of R1 (round 1, kappa < 8) and R2 (round 2, kappa >= 8) of
    lane q of 16-lane group s of wave w; R1[i] pairs with R2[15 - i] except on
    the special lane."""
    if w == 0 and s == 0:
        # column 0 (pair 0): the special lane q = 0 holds (0, 0) and (0, 8),
        # lanes q = 1..7 (0, q) <-> (0, 16 - q); column 16 (pair 1) on lanes
        # q = 8..15: (16, q - 8) <-> (16, 23 - q).  Lane q's R1 slot is q mod
        # 16, so the group's T2 reads stay conflict-free
        if q == 0:
            return (0, 0), (0, 8)
        if q < 8:
            return (0, q), (0, 16 - q)
        return (1, q - 8), (1, 23 - q)
    if q < 8:
        return (0, q), (1, 15 - q)
    return (1, q - 8), (0, 15 - (q - 8))


SPECIAL = (0, 0, 0)  # (w, s, q): lane 0 of wave 0

# ---- bank-conflict checks (as scripts/fft32r_model.py) ------------------------
RD_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)],
             [*range(4, 12), *range(16, 20), *range(28, 32)]]
RD_GROUPS += [[l + 32 for l in grp] for grp in RD_GROUPS]
WRITE_CONFLICTS = []


def check_write(slots, what):
    extra = 0
    for g in range(8):
        grp = [slots[l] % 8 for l in range(8 * g, 8 * g + 8) if slots[l] is not None]
        extra += max(grp.count(v) for v in set(grp)) - 1
    if extra:
        WRITE_CONFLICTS.append((what, extra))


def check_read(slots, what, conflicts):
    for grp in RD_GROUPS:
        vals = [slots[l] for l in grp if slots[l] is not None]
        m = [v % 16 for v in vals]
        ways = max(m.count(v) for v in set(m)) if m else 1
        if ways > 1:
            conflicts.append((what, ways))


class Lds:
    def __init__(self):
        self.v = np.full(NW * RG, np.nan + 1j * np.nan)
        self.tag = [None] * (NW * RG)

    def write(self, slot, val, tag):
        assert 0 <= slot < NW * RG
        self.v[slot] = val
        self.tag[slot] = tag

    def read(self, slot, tag):
        assert self.tag[slot] == tag, (slot, self.tag[slot], tag)
        return self.v[slot]


# ---- LDS layouts --------------------------------------------------------------
def t1_slot(b, k1):
    """T1 image of thread b's register k1 (either round: k1 mod 16): each wave
    writes its own region, 64 consecutive threads per register row"""
    return RG * (b >> 6) + 64 * (k1 & 15) + (b & 63)


def t2_slot(w, s, pair, kl, gamma):
    """T2 image (either round): wave w's region, 16-lane group s, pair, local
    kappa kl < 8, gamma; rows of 17 slots"""
    return RG * w + 272 * s + 136 * pair + 17 * kl + gamma


def dft(v, axis=-1):
    return np.fft.fft(v, axis=axis)


def W(n, e):
    return np.exp(-2j * np.pi * np.asarray(e, dtype=np.float64) / n)


def pair_tables(taps):
    """zero-phase pair coefficients p1, q2, p2 per bin k of the N-point
    transform (fir_fft.hpp's r16_plan_tables)"""
    T = len(taps)
    half = (T - 1) // 2
    g = np.zeros(L)
    for j in range(-half, half + 1):
        g[j % L] = 0.5 * (taps[half + j] + taps[half - j])
    G = np.fft.fft(g) / (4.0 * N)
    k = np.arange(N)
    Gk, Gm = G[k], np.conj(G[(N - k) % L])
    Sv, Dv = Gk + Gm, Gk - Gm
    wv = W(L, k)
    p1 = 2 * Sv.real + 2 * Dv.real * wv.imag
    q2 = 2 * Sv.real - 2 * Dv.real * wv.imag
    p2 = 2 * Dv.real * wv.real
    c8 = 2 * Sv.real[N // 2] - 2 * Dv.real[N // 2]
    return p1, q2, p2, c8


def pair_sym(P, Q, p1, q2, p2):
    oP = np.conj(P * p1 + np.conj(Q) * 1j * p2)
    oQ = np.conj(Q) * q2 - P * 1j * p2
    return oP, oQ


def bin_of(k1, kap, lam):
    return k1 + 32 * kap + 512 * lam


def run(taps, x_seg, tables=None):
    """One unit on segment x_seg.  tables: the host's plan tables (task words,
    pair coefficients per (thread, slot), c8) instead of this model's own."""
    conflicts = []
    tasks = t2_tasks
    if tables is not None:
        def tasks(w, s, q):  # noqa: F811  (r16_task_word's bit fields)
            tk = int(tables["task"][64 * w + 16 * s + q])
            return (tk & 1, (tk >> 1) & 7), ((tk >> 4) & 1, 8 + ((tk >> 5) & 7))
    z = x_seg[0::2] + 1j * x_seg[1::2]
    # ---- stage 1: thread b, register n -> k1
    reg1 = {}
    for b in range(NT):
        a = np.array([z[256 * n + b] for n in range(32)])
        reg1[b] = dft(a) * W(N, b * np.arange(32))
    col = {}  # (k1, gamma) -> 16 values, beta = 0..15
    for rnd in range(2):
        # ---- T1 round rnd: thread b writes registers 16 rnd .. 16 rnd + 15
        lds = Lds()
        for w in range(NW):
            for i in range(16):
                slots = []
                for lane in range(64):
                    b = 64 * w + lane
                    k1 = 16 * rnd + i
                    s_ = t1_slot(b, k1)
                    lds.write(s_, reg1[b][k1], ("t1", b, k1))
                    slots.append(s_)
                check_write(slots, f"T1w r{rnd} w{w}")
        # lane (w, s, gamma) reads column pair_cols(w, s)[rnd], beta = i
        for w in range(NW):
            for i in range(16):
                slots = []
                for lane in range(64):
                    s, gamma = lane >> 4, lane & 15
                    k1 = pair_cols(w, s)[rnd]
                    # column 16 (wave 0, group 0, pair B) sits in round 1's
                    # rows: k1 16..31 map to rows 0..15
                    assert (k1 >= 16) == (rnd == 1)
                    b = 16 * i + gamma
                    s_ = t1_slot(b, k1)
                    col.setdefault((k1, gamma), [None] * 16)[i] = lds.read(s_, ("t1", b, k1))
                    slots.append(s_)
                check_read(slots, f"T1r r{rnd} w{w}", conflicts)
    # ---- stage 2: DFT16 over beta -> kappa, * W_256^(gamma kappa)
    inner = {}
    for (k1, gamma), v in col.items():
        inner[(k1, gamma)] = dft(np.array(v)) * W(256, gamma * np.arange(16))
    # ---- T2, two rounds (kappa < 8, kappa >= 8) per wave
    R = {}
    for w in range(NW):
        for rnd in range(2):
            lds = Lds()
            for kl in range(8):
                for pair in range(2):
                    slots = []
                    for lane in range(64):
                        s, gamma = lane >> 4, lane & 15
                        k1 = pair_cols(w, s)[pair]
                        kap = 8 * rnd + kl
                        sl = t2_slot(w, s, pair, kl, gamma)
                        lds.write(sl, inner[(k1, gamma)][kap], ("t2", k1, kap, gamma))
                        slots.append(sl)
                    check_write(slots, f"T2w w{w} r{rnd}")
            for i in range(16):  # register i = gamma
                slots = []
                for lane in range(64):
                    s, q = lane >> 4, lane & 15
                    pair, kap = tasks(w, s, q)[rnd]
                    assert (kap >= 8) == (rnd == 1)
                    k1 = pair_cols(w, s)[pair]
                    sl = t2_slot(w, s, pair, kap - 8 * rnd, i)
                    R.setdefault((w, s, q), [[None] * 16, [None] * 16])[rnd][i] = lds.read(
                        sl, ("t2", k1, kap, i))
                    slots.append(sl)
                check_read(slots, f"T2r w{w} r{rnd}", conflicts)
    # ---- stage 3 and the spectrum check
    Zref = np.fft.fft(z)
    err = 0.0
    for (w, s, q), (r1, r2) in R.items():
        for rnd, reg in enumerate((r1, r2)):
            out = dft(np.array(reg))
            R[(w, s, q)][rnd] = out
            pair, kap = tasks(w, s, q)[rnd]
            k1 = pair_cols(w, s)[pair]
            err = max(err, np.max(np.abs(out - Zref[bin_of(k1, kap, np.arange(16))])))
    assert err < 1e-6 * np.max(np.abs(Zref)), err
    # ---- pair step
    p1, q2, p2, c8 = pair_tables(taps) if tables is None else (None, None, None, tables["c8"][0].real)

    def coef(t, i, k):
        if tables is None:
            return p1[k], q2[k], p2[k]
        pq = tables["pair"][i * NT + t]
        pp = tables["pair"][(16 + i // 2) * NT + t]
        return pq.real, pq.imag, (pp.imag if i & 1 else pp.real)
    for (w, s, q), (r1, r2) in R.items():
        x, y = list(r1), list(r2)
        (pa, kap1), (pb, kap2) = tasks(w, s, q)
        bx = [bin_of(pair_cols(w, s)[pa], kap1, lam) for lam in range(16)]
        by = [bin_of(pair_cols(w, s)[pb], kap2, lam) for lam in range(16)]
        special = (w, s, q) == SPECIAL
        if special:
            v8, b8 = x[8], bx[8]
            x, y, bx, by = (y[0:8] + x[1:8] + [x[0]], [x[0]] + x[9:16] + y[8:16],
                            by[0:8] + bx[1:8] + [bx[0]], [bx[0]] + bx[9:16] + by[8:16])
            assert b8 == N // 2
        for i in range(16):
            kP, kQ = bx[i], by[15 - i]
            assert (kP + kQ) % N == 0, (w, s, q, i, kP, kQ)
            x[i], y[15 - i] = pair_sym(x[i], y[15 - i], *coef(64 * w + 16 * s + q, i, kP))
        if special:
            o8 = np.conj(v8 * c8)
            r1n = [x[15]] + x[8:15] + [o8] + y[1:8]
            r2n = x[0:8] + y[8:16]
            x, y = r1n, r2n
        R[(w, s, q)] = [x, y]
    # ---- inverse stage 3
    for key, (r1, r2) in R.items():
        R[key] = [dft(np.array(r1)), dft(np.array(r2))]
    # ---- T2': task lanes write, (pair, gamma) lanes gather kappa
    colk = {}
    for w in range(NW):
        for rnd in range(2):
            lds = Lds()
            for i in range(16):
                slots = []
                for lane in range(64):
                    s, q = lane >> 4, lane & 15
                    pair, kap = tasks(w, s, q)[rnd]
                    sl = t2_slot(w, s, pair, kap - 8 * rnd, i)
                    lds.write(sl, R[(w, s, q)][rnd][i], ("t2i", w, s, pair, kap, i))
                    slots.append(sl)
                check_write(slots, f"T2'w w{w} r{rnd}")
            for kl in range(8):
                for pair in range(2):
                    slots = []
                    for lane in range(64):
                        s, gamma = lane >> 4, lane & 15
                        kap = 8 * rnd + kl
                        sl = t2_slot(w, s, pair, kl, gamma)
                        colk.setdefault((pair_cols(w, s)[pair], gamma), [None] * 16)[kap] = lds.read(
                            sl, ("t2i", w, s, pair, kap, gamma))
                        slots.append(sl)
                    check_read(slots, f"T2'r w{w} r{rnd}", conflicts)
    # ---- stage 2': * W_256^(gamma kappa), DFT16 over kappa -> beta
    U2 = {}
    for (k1, gamma), v in colk.items():
        U2[(k1, gamma)] = dft(np.array(v) * W(256, gamma * np.arange(16)))
    # ---- T1': round rnd carries pair rnd back; thread b reads k1 = 16 rnd + r
    fin = {b: [None] * 32 for b in range(NT)}
    for rnd in range(2):
        lds = Lds()
        for w in range(NW):
            for i in range(16):
                slots = []
                for lane in range(64):
                    s, gamma = lane >> 4, lane & 15
                    k1 = pair_cols(w, s)[rnd]
                    b = 16 * i + gamma
                    s_ = t1_slot(b, k1)
                    lds.write(s_, U2[(k1, gamma)][i], ("t1i", b, k1))
                    slots.append(s_)
                check_write(slots, f"T1'w r{rnd} w{w}")
        for w in range(NW):
            for r in range(16):
                slots = []
                for lane in range(64):
                    b = 64 * w + lane
                    k1 = 16 * rnd + r
                    s_ = t1_slot(b, k1)
                    fin[b][k1] = lds.read(s_, ("t1i", b, k1))
                    slots.append(s_)
                check_read(slots, f"T1'r r{rnd} w{w}", conflicts)
    # ---- final: * W_N^(b k1), DFT32 over k1 -> n; out[256 n + b]
    out = np.zeros(N, complex)
    for b in range(NT):
        v = dft(np.array(fin[b]) * W(N, b * np.arange(32)))
        out[256 * np.arange(32) + b] = v
    c = np.empty(L)
    c[0::2] = out.real
    c[1::2] = -out.imag
    return c, conflicts


def main(ntaps=None):
    if ntaps is None:
        ntaps = int(sys.argv[1]) if len(sys.argv) > 1 else 4001
    rng = np.random.default_rng(5)
    half = (ntaps - 1) // 2
    n = np.arange(ntaps) - half
    taps = np.sinc(n / 400.0) * np.hanning(ntaps)  # symmetric
    taps /= taps.sum()
    x_seg = rng.standard_normal(L)
    c, conflicts = run(taps, x_seg)
    ref = np.array([np.dot(taps, x_seg[m - half:m + half + 1]) for m in range(half, L - half, 997)])
    got = c[half:L - half:997]
    err = np.max(np.abs(got - ref))
    print(f"ntaps {ntaps}: max |err| {err:.3e} over {len(ref)} outputs; read conflicts: "
          f"{sorted(set(conflicts)) if conflicts else 'none'}; write extra cycles: "
          f"{sorted(set(WRITE_CONFLICTS)) if WRITE_CONFLICTS else 'none'}")
    assert err < 1e-10, err


if __name__ == "__main__":
    main()

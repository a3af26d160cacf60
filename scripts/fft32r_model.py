#!/usr/bin/env python3
"""numpy model of the register-resident L = 32 768 overlap-save unit
(csrc/fir_fft32r.hpp), zero-phase form.  It runs the kernel's data flow thread
by thread -- every register index, LDS slot and pair-table slot -- and checks

  * each LDS exchange round: every slot written once, every read gets the
    value the index algebra says, b128 stores conflict-free in their 8-lane
    groups and b128 loads in their 16-lane groups (MI355X_MICROARCH.md, LDS);
  * the forward spectrum after stage 3 against numpy's FFT;
  * the outputs against a direct convolution.

The transform: N = 16 384 complex points z[m] = x_seg[2m] + i x_seg[2m+1],
m = 512 a + b (thread b of 512, register a of 32), b = 16 beta + gamma.
  stage 1 (thread b): DFT32 over a -> k1, * W_N^(b k1); waves 4..7 negate the
     odd inputs, so register r holds k1 = r + 16 (mod 32) there
  T1 (workgroup, 2 rounds: registers 0..15, then 16..31): column k1's 16
     lanes gamma gather beta = 0..31 (rotated by 16 for k1 >= 16)
  stage 2 (lane (k1, gamma)): DFT32 over beta -> kappa, * W_512^(gamma kappa)
  T2 (wave-local, 2 rounds): lane s of a 32-lane group gathers gamma for
     two tasks (column, kappa), one per round (R1, R2)
  stage 3: DFT16 over gamma -> lambda:  Z[k1 + 32 kappa + 1024 lambda]
  pair step (R1[i] with R2[15 - i]), then the same stages backwards.
usage: fft32r_model.py [ntaps]     the data-flow model
       fft32r_model.py --price     price structural changes of the unit (price())
"""
import sys

import numpy as np

N = 16384
L = 2 * N
NT = 512

# ---- column ownership -------------------------------------------------------
# wave w, 32-lane group g, half h (16 lanes each) -> column k1
def column(w, g, h):
    if w == 0:
        return [[0, 16], [8, 24]][g][h]
    return [[w, 32 - w], [w + 8, 24 - w]][g][h]


COL_OF = {}  # k1 -> (w, g, h)
for w in range(8):
    for g in range(2):
        for h in range(2):
            COL_OF[column(w, g, h)] = (w, g, h)
assert sorted(COL_OF) == list(range(32))
# ---- T2 task assignment ---------------------------------------------------------
def t2_tasks(w, g, s):
    """(h, kappa) of R1 (round 1, kappa < 16) and R2 (round 2, kappa >= 16) of
    lane s in group g of wave w; R1[i] pairs with R2[15 - i] except in the
    special group (wave 0, g = 0: columns 0 and 16)."""
    if w == 0 and g == 0:
        # column 16's tasks (16, k) <-> (16, 31 - k) on the lanes of read group
        # GA = {0-3, 12-15, 20-27}, column 0's (0, k) <-> (0, 32 - k), k = 1..15,
        # and the special lane on GB: distinct kappa_local in every read group
        # and round (conflict-free T2 reads)
        ga = [*range(0, 4), *range(12, 16), *range(20, 28)]
        if s in ga:
            kap = ga.index(s)
            return (1, kap), (1, 31 - kap)
        if s < 31:
            gb = [*range(4, 12), *range(16, 20), *range(28, 31)]
            kap = 1 + gb.index(s)
            return (0, kap), (0, 32 - kap)
        return (0, 0), (0, 16)  # the special lane: both self-paired
    if s < 16:
        return (0, s), (1, 31 - s)
    return (1, 31 - s), (0, s)


SPECIAL = (0, 0, 31)  # (w, g, s) of the special lane: lane 31 of wave 0

# ---- bank-conflict checks (MI355X_MICROARCH.md LDS table) -------------------------
RD_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)],
             [*range(4, 12), *range(16, 20), *range(28, 32)]]
RD_GROUPS += [[l + 32 for l in grp] for grp in RD_GROUPS]


WRITE_CONFLICTS = []


def check_write(slots, what):
    """slots[lane] (16-B units) of one ds_write_b128 of a wave: 8 lane groups
    of 8, bank (a/4) mod 32 -> slots distinct mod 8 in a group.  Extra LDS-array
    cycles are recorded; a b128 store costs ~13 cycles of transfer against 8
    array cycles, so a few extra array cycles per instruction are free."""
    extra = 0
    for q in range(8):
        grp = [slots[l] % 8 for l in range(8 * q, 8 * q + 8) if slots[l] is not None]
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


# ---- the LDS image ----------------------------------------------------------------
class Lds:
    def __init__(self):
        self.v = np.full(8 * RG, np.nan + 1j * np.nan)
        self.tag = [None] * (8 * RG)

    def write(self, slot, val, tag):
        assert 0 <= slot < 8 * RG
        self.v[slot] = val
        self.tag[slot] = tag

    def read(self, slot, tag):
        assert self.tag[slot] == tag, (slot, self.tag[slot], tag)
        return self.v[slot]


# T2 (wave-local, both rounds): (g, h, kappa_local, gamma) in wave w's region
# the kernel's LDS layout (fir_fft32r.hpp, LCFIR_R32_PAD = 1): one region of
# RG slots per wave; T2 rows padded to 17 slots (a reader's addresses are its
# row base + register index, conflict-free without a swizzle)
PAD = True
RG = 1088 if PAD else 1024


def t2_slot(w, g, h, kl, gamma):
    if PAD:
        return RG * w + 544 * g + 272 * h + 17 * kl + gamma
    return RG * w + 512 * g + 256 * h + 16 * kl + (gamma ^ kl)


def dft(v, axis=-1):
    return np.fft.fft(v, axis=axis)


def W(n, e):
    return np.exp(-2j * np.pi * np.asarray(e, dtype=np.float64) / n)


def pair_tables(taps):
    """zero-phase pair coefficients p1, q2, p2 per bin k of the N-point
    transform (fir_fft.hpp's fft_plan_tables for L = 32 768, halves = 1)"""
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
    return k1 + 32 * kap + 1024 * lam


def run(taps, x_seg, tables=None):
    """One unit of the kernel on segment x_seg.  tables: the host's plan
    tables (fft_tables_dump, fft32_model.load_tables) -- task words, pair
    coefficients per (thread, slot) and c8 -- instead of this model's own."""
    conflicts = []
    tasks = t2_tasks
    if tables is not None:
        def tasks(w, g, s):  # noqa: F811  (r32_task_word's bit fields)
            tk = int(tables["task"][64 * w + 32 * g + s])
            return (tk & 1, (tk >> 1) & 15), ((tk >> 5) & 1, 16 + ((tk >> 6) & 15))
    z = x_seg[0::2] + 1j * x_seg[1::2]
    # ---- stage 1: thread b, register n; waves 4..7 (sigma = 1) negate the odd
    # inputs, so register r holds k1 = (r + 16 sigma) mod 32: registers 0..15
    # are the round-1 columns of every thread (k1 < 16 iff b < 256)
    def k1_of(r, sig):
        return (r + 16 * sig) % 32
    reg1 = {}
    for b in range(NT):
        sig = int(b >= 256)
        a = np.array([z[512 * n + b] * (-1) ** (n * sig) for n in range(32)])
        A = dft(a)
        reg1[b] = A * W(N, b * np.array([k1_of(r, sig) for r in range(32)]))
    # ---- T1 round 1: thread b writes registers 0..15 into its own region;
    # lane (k1, gamma) reads beta = i + 16 h into c[i]
    lds = Lds()
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                b = 64 * w + lane
                s_ = RG * w + 64 * i + lane
                lds.write(s_, reg1[b][i], ("t1", b, k1_of(i, int(b >= 256))))
                slots.append(s_)
            check_write(slots, f"T1w1 w{w} i{i}")
    col = {}  # (k1, gamma) -> c[n], n = 0..31, holding beta = (n + 16 h) mod 32
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                g, h, gamma = lane >> 5, (lane >> 4) & 1, lane & 15
                k1 = column(w, g, h)
                assert (k1 >= 16) == bool(h)
                beta = i + 16 * h
                b = 16 * beta + gamma
                s_ = RG * (b >> 6) + 64 * (k1 & 15) + (b & 63)
                col.setdefault((k1, gamma), [None] * 32)[i] = lds.read(s_, ("t1", b, k1))
                slots.append(s_)
            check_read(slots, f"T1r1 w{w}", conflicts)
    # ---- T1 round 2: registers 16..31 into the reader's region
    lds = Lds()
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                b = 64 * w + lane
                k1 = k1_of(16 + i, int(b >= 256))
                cw, cg, ch = COL_OF[k1]
                s_ = RG * cw + 256 * (2 * cg + ch) + 16 * ((b >> 4) & 15) + (b & 15)
                lds.write(s_, reg1[b][16 + i], ("t1", b, k1))
                slots.append(s_)
            check_write(slots, f"T1w2 w{w} i{i}")
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                g, h, gamma = lane >> 5, (lane >> 4) & 1, lane & 15
                k1 = column(w, g, h)
                beta = i + 16 * (1 - h)
                b = 16 * beta + gamma
                s_ = RG * w + 256 * (2 * g + h) + 16 * i + gamma
                col[(k1, gamma)][16 + i] = lds.read(s_, ("t1", b, k1))
                slots.append(s_)
            check_read(slots, f"T1r2 w{w}", conflicts)
    # ---- stage 2: DFT32 over n (beta rotated by 16 h: the output picks up
    # (-1)^(kappa h)), * (s W_512^gamma)^kappa with s = (-1)^h: natural order
    inner = {}
    for (k1, gamma), v in col.items():
        h = COL_OF[k1][2]
        base = (-1) ** h * W(512, gamma)
        inner[(k1, gamma)] = dft(np.array(v)) * base ** np.arange(32)
    # ---- T2, two rounds per wave
    R = {}  # (w, g, s) -> [R1 (16), R2 (16)]
    for w in range(8):
        for rnd in range(2):
            lds = Lds()
            for kl in range(16):
                slots = []
                for lane in range(64):
                    g, h, gamma = lane >> 5, (lane >> 4) & 1, lane & 15
                    k1 = column(w, g, h)
                    kap = 16 * rnd + kl
                    s = t2_slot(w, g, h, kl, gamma)
                    lds.write(s, inner[(k1, gamma)][kap], ("t2", k1, kap, gamma))
                    slots.append(s)
                check_write(slots, f"T2w w{w} r{rnd}")
            for i in range(16):  # register i = gamma
                slots = []
                for lane in range(64):
                    g, s_ = lane >> 5, lane & 31
                    h, kap = tasks(w, g, s_)[rnd]
                    assert (kap >= 16) == (rnd == 1)
                    k1 = column(w, g, h)
                    s = t2_slot(w, g, h, kap - 16 * rnd, i)
                    R.setdefault((w, g, s_), [[None] * 16, [None] * 16])[rnd][i] = lds.read(
                        s, ("t2", k1, kap, i))
                    slots.append(s)
                check_read(slots, f"T2r w{w} r{rnd}", conflicts)
    # ---- stage 3: DFT16 over gamma -> lambda; check the spectrum
    Zref = np.fft.fft(z)
    err = 0.0
    for (w, g, s_), (r1, r2) in R.items():
        for rnd, reg in enumerate((r1, r2)):
            out = dft(np.array(reg))
            R[(w, g, s_)][rnd] = out
            h, kap = tasks(w, g, s_)[rnd]
            k1 = column(w, g, h)
            err = max(err, np.max(np.abs(out - Zref[bin_of(k1, kap, np.arange(16))])))
    assert err < 1e-6 * np.max(np.abs(Zref)), err
    # ---- pair step: slot i pairs P = x[i], Q = y[15 - i]; table by P's bin
    p1, q2, p2, c8 = pair_tables(taps) if tables is None else (None, None, None, tables["c8"][0].real)

    def coef(t, i, k):
        if tables is None:
            return p1[k], q2[k], p2[k]
        pq = tables["pair"][i * NT + t]
        pp = tables["pair"][(16 + i // 2) * NT + t]
        return pq.real, pq.imag, (pp.imag if i & 1 else pp.real)
    for (w, g, s_), (r1, r2) in R.items():
        x, y = list(r1), list(r2)
        (h1, kap1), (h2, kap2) = tasks(w, g, s_)
        bx = [bin_of(column(w, g, h1), kap1, lam) for lam in range(16)]
        by = [bin_of(column(w, g, h2), kap2, lam) for lam in range(16)]
        special = (w, g, s_) == SPECIAL
        if special:
            # x' = [R2[0..7], R1[1..7], R1[0]], y' = [R1[0], R1[9..15], R2[8..15]]; R1[8] apart
            v8, b8 = x[8], bx[8]
            x, y, bx, by = (y[0:8] + x[1:8] + [x[0]], [x[0]] + x[9:16] + y[8:16],
                            by[0:8] + bx[1:8] + [bx[0]], [bx[0]] + bx[9:16] + by[8:16])
            assert b8 == N // 2
        for i in range(16):
            kP, kQ = bx[i], by[15 - i]
            assert (kP + kQ) % N == 0, (w, g, s_, i, kP, kQ)
            x[i], y[15 - i] = pair_sym(x[i], y[15 - i], *coef(64 * w + 32 * g + s_, i, kP))
        if special:
            o8 = np.conj(v8 * c8)
            # inverse permutation (slot 15's Q output, a duplicate of bin 0's, is dropped)
            r1n = [x[15]] + x[8:15] + [o8] + y[1:8]
            r2n = x[0:8] + y[8:16]
            x, y = r1n, r2n
        R[(w, g, s_)] = [x, y]
    # ---- inverse stage 3': DFT16 over lambda -> gamma (on conj(V))
    for key, (r1, r2) in R.items():
        R[key] = [dft(np.array(r1)), dft(np.array(r2))]
    # ---- T2': writers lane s (register gamma), readers (h, gamma) gather kappa
    colk = {}
    for w in range(8):
        for rnd in range(2):
            lds = Lds()
            for i in range(16):
                slots = []
                for lane in range(64):
                    g, s_ = lane >> 5, lane & 31
                    h, kap = tasks(w, g, s_)[rnd]
                    s = t2_slot(w, g, h, kap - 16 * rnd, i)
                    lds.write(s, R[(w, g, s_)][rnd][i], ("t2i", w, g, h, kap, i))
                    slots.append(s)
                check_write(slots, f"T2'w w{w} r{rnd}")
            for kl in range(16):
                slots = []
                for lane in range(64):
                    g, h, gamma = lane >> 5, (lane >> 4) & 1, lane & 15
                    kap = 16 * rnd + kl
                    s = t2_slot(w, g, h, kl, gamma)
                    colk.setdefault((column(w, g, h), gamma), [None] * 32)[kap] = lds.read(
                        s, ("t2i", w, g, h, kap, gamma))
                    slots.append(s)
                check_read(slots, f"T2'r w{w} r{rnd}", conflicts)
    # ---- stage 2': * (s W_512^gamma)^kappa, DFT32 over kappa: c[n] holds
    # beta = (n + 16 h) mod 32
    U2 = {}
    for (k1, gamma), v in colk.items():
        h = COL_OF[k1][2]
        base = (-1) ** h * W(512, gamma)
        U2[(k1, gamma)] = dft(np.array(v) * base ** np.arange(32))
    # ---- T1' round 1: registers 0..15 into the writer's region; thread b reads
    # k1 = r + 16 sigma into fin[r]
    fin = {b: [None] * 32 for b in range(NT)}
    lds = Lds()
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                g, h, gamma = lane >> 5, (lane >> 4) & 1, lane & 15
                k1 = column(w, g, h)
                beta = i + 16 * h
                s_ = RG * w + 64 * i + lane
                lds.write(s_, U2[(k1, gamma)][i], ("t1i", 16 * beta + gamma, k1))
                slots.append(s_)
            check_write(slots, f"T1'w1 w{w}")
    for w in range(8):
        for r in range(16):
            slots = []
            for lane in range(64):
                b = 64 * w + lane
                sig = int(b >= 256)
                k1 = k1_of(r, sig)
                cw, cg, ch = COL_OF[k1]
                beta, gamma = b >> 4, b & 15
                s_ = RG * cw + 64 * (beta & 15) + 32 * cg + 16 * ch + gamma
                fin[b][r] = lds.read(s_, ("t1i", b, k1))
                slots.append(s_)
            check_read(slots, f"T1'r1 w{w}", conflicts)
    # ---- T1' round 2: registers 16..31 into the reader's region
    lds = Lds()
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                g, h, gamma = lane >> 5, (lane >> 4) & 1, lane & 15
                k1 = column(w, g, h)
                beta = (16 + i + 16 * h) % 32
                b = 16 * beta + gamma
                s_ = RG * (b >> 6) + 64 * (k1 & 15) + (b & 63)
                lds.write(s_, U2[(k1, gamma)][16 + i], ("t1i", b, k1))
                slots.append(s_)
            check_write(slots, f"T1'w2 w{w}")
    for w in range(8):
        for i in range(16):
            slots = []
            for lane in range(64):
                b = 64 * w + lane
                k1 = k1_of(16 + i, int(b >= 256))
                s_ = RG * w + 64 * i + lane
                fin[b][16 + i] = lds.read(s_, ("t1i", b, k1))
                slots.append(s_)
            check_read(slots, f"T1'r2 w{w}", conflicts)
    # ---- final: * W_N^(b k1), DFT32 over r -> a (times (-1)^(a sigma)); out[512 a + b]
    out = np.zeros(N, complex)
    for b in range(NT):
        sig = int(b >= 256)
        k1s = np.array([k1_of(r, sig) for r in range(32)])
        v = dft(np.array(fin[b]) * W(N, b * k1s))
        v = v * (-1.0) ** (np.arange(32) * sig)
        out[512 * np.arange(32) + b] = v
    c = np.empty(L)
    c[0::2] = out.real
    c[1::2] = -out.imag
    return c, conflicts


# ---- pricing structural changes of the unit -----
# Measured inputs, each from a committed file:
#   unit and phase cycles: profiles/r06_pricing/trace_prod.log (config 2, 4 001 taps,
#     tools/fft32r_trace.hip: per-wave s_memtime at every phase boundary, this tree)
#   the next unit's staging DMA, priced by removing it: scripts/variants/nodma.patch
#     (timing only, stale samples), alternating with the product on one box,
#     profiles/r06_pricing/ab_prod_nodma.txt (launch 0.1779 -> 0.1623 ms) and its trace
#     profiles/r06_pricing/trace_nodma.log
#   the whole memory phase, priced by removing the DMA and the output stores:
#     scripts/variants/nodma_nostore.patch, three-way alternation on one box,
#     profiles/r06_pricing/ab_prod_nodma_nostore.txt
#   barrier costs: the trace's BAR2 / BAR5 (barriers that follow a round, not the first
#     of an exchange, which absorbs the older / younger waves' skew)
#   LDS: MI355X_MICROARCH.md "LDS"; capacities from fir_fft32r.hpp (kR32Work, kR32Tw)
PRICE = {
    "unit_cycles": (58.9e3 + 60.3e3) / 2,   # older / younger waves' unit total (trace_prod.log)
    "launch_ms": (0.177865 + 0.178027 + 0.178767) / 3,       # product, ab_prod_nodma.txt
    "launch_nodma_ms": (0.162609 + 0.162073 + 0.162253) / 3,  # no staging DMA at all (timing only)
    # prod / no DMA / neither, alternating (ab_prod_nodma_nostore.txt)
    "ab3_launch_ms": (0.18036 + 0.179066 + 0.17924) / 3,
    "ab3_nodma_ms": (0.162822 + 0.162772 + 0.1631) / 3,
    "ab3_nomem_ms": (0.160374 + 0.160546 + 0.160434) / 3,
    "round_barrier_cycles": (667 + 691) / 2,  # BAR2, BAR5 (r05 trace; r06's within 3 %)
    "lds_round_trip_cycles": 500,           # one exposed write -> read latency of a wave-local round
    "lds_bytes": 160 * 1024,
    "dma_bytes": 128 * 1024,                # the next unit's samples (32 768 f32)
    "work_array_bytes": 8 * 1088 * 16,      # kR32Work double2 (T1 / T2 / T2' / T1' and the staged samples)
    "twiddle_bytes": (1024 + 16 + 2 + 32) * 16,  # kR32Tw + peak slots + the special lane's scratch
}
BUILD_BAR = 0.08


def memory_phase_ceiling():
    """(no-DMA gain, no-DMA-and-no-stores gain) of the three-way alternation:
    what any change to the unit's HBM traffic can take at most."""
    P = PRICE
    return 1.0 - P["ab3_nodma_ms"] / P["ab3_launch_ms"], 1.0 - P["ab3_nomem_ms"] / P["ab3_launch_ms"]


def price(verbose=True):
    """Price the candidate changes of fir_fft32r's unit against the product.
    Returns {design: (feasible, net gain, best-case gain)} as fractions of the
    launch (negative: slower); the build bar is a net gain >= BUILD_BAR.

    The ceiling of every design that moves staging traffic out of the final
    phase is measured, not modelled: the product with no staging DMA at all
    (scripts/variants/nodma.patch, timing only) runs 8.8 % faster.  A design
    gets at most its share of that; its extra barriers and exposed LDS
    rounds are charged at the trace's costs."""
    P = PRICE
    ceiling = 1.0 - P["launch_nodma_ms"] / P["launch_ms"]
    unit = P["unit_cycles"]
    free_lds = P["lds_bytes"] - P["work_array_bytes"] - P["twiddle_bytes"]
    out, lines = {}, []
    lines.append(f"ceiling (no staging DMA at all, timing only): launch {P['launch_ms']:.4f} -> "
                 f"{P['launch_nodma_ms']:.4f} ms = {100 * ceiling:.1f} % (build bar {100 * BUILD_BAR:.0f} %)")
    # (B) half of the next unit's samples staged early: T2' and T1' in 4 rounds
    # of 64 KiB so that half of every wave's region is free from T2' on; that
    # half's DMA issued after T2', the rest in the final phase as now
    best_b = ceiling / 2
    cost_b = (4 * P["round_barrier_cycles"] + 4 * P["lds_round_trip_cycles"]) / unit
    out["half_dma_early"] = (True, best_b - cost_b, best_b)
    lines.append(f"(B) half the DMA early (T2' and T1' in 4 rounds of 64 KiB): at most {100 * best_b:.1f} %; "
                 f"+4 barriers and +4 exposed rounds cost {100 * cost_b:.1f} %: net {100 * (best_b - cost_b):+.1f} %")
    # (C) all of it early: the 128 KiB of samples must coexist with T1''s rounds
    room = P["lds_bytes"] - P["dma_bytes"] - P["twiddle_bytes"]
    rounds_c = int(np.ceil(256 * 1024 / room))
    cost_c = (2 * (rounds_c - 2) * P["round_barrier_cycles"] + (rounds_c - 2) * P["lds_round_trip_cycles"]) / unit
    out["all_dma_early"] = (True, ceiling - cost_c, ceiling)
    lines.append(f"(C) all of it early: {room / 1024:.1f} KiB of LDS beside the samples -> T1' in {rounds_c} rounds "
                 f"(+{2 * (rounds_c - 2)} barriers): at most {100 * ceiling:.1f} %, costs {100 * cost_c:.1f} %: "
                 f"net {100 * (ceiling - cost_c):+.1f} %")
    # (D) the final phase's twiddles W_16384^(b k1) from an LDS table: whole,
    # 512 x 32 x 16 B; factored W_1024^(beta k1) W_16384^(gamma k1), 24 KiB,
    # but one complex product per power (4 f64 ops) more, against the anchored
    # chain's 3 per power it replaces
    tab_full, tab_fact = 512 * 32 * 16, (32 * 32 + 16 * 32) * 16
    out["final_twiddles_lds"] = (tab_fact <= free_lds, -(4 - 3) * 32 * 2 * 4.1 / unit, 0.0)
    lines.append(f"(D) final twiddles from an LDS table: {tab_full // 1024} KiB whole / {tab_fact // 1024} KiB "
                 f"factored against {free_lds / 1024:.1f} KiB free beside the work array and the twiddles; "
                 f"the factored form costs 4 f64 ops per power against the chain's 3: no gain even with room")
    dma3, mem3 = memory_phase_ceiling()
    lines.append(f"ceiling of the whole memory phase (no DMA and no output stores, timing only): "
                 f"{100 * mem3:.1f} % (no DMA alone {100 * dma3:.1f} % in the same alternation): "
                 f"no memory-side change of the unit can take more")
    if verbose:
        print("\n".join(lines))
    return out


def main(ntaps=None):
    if ntaps is None:
        if len(sys.argv) > 1 and sys.argv[1] == "--price":
            price()
            return
        ntaps = int(sys.argv[1]) if len(sys.argv) > 1 else 8001
    rng = np.random.default_rng(5)
    half = (ntaps - 1) // 2
    n = np.arange(ntaps) - half
    taps = np.sinc(n / 400.0) * np.hanning(ntaps)  # symmetric
    taps /= taps.sum()
    x_seg = rng.standard_normal(L)
    c, conflicts = run(taps, x_seg)
    # zero-phase: c[m] = sum_j h[half + j] x_seg[m - j]?  check against the
    # direct form on the valid range m in [half, L - half)
    ref = np.convolve(x_seg, taps[::-1], mode="full")  # ref[m + ntaps - 1 - ...]
    # y[m] = sum_k h[k] x_seg[m - half + k]  (FilterCore.h's window, centred)
    ref = np.array([np.dot(taps, x_seg[m - half:m + half + 1]) for m in range(half, L - half, 997)])
    got = c[half:L - half:997]
    err = np.max(np.abs(got - ref))
    print(f"ntaps {ntaps}: max |err| {err:.3e} over {len(ref)} outputs; read conflicts: "
          f"{sorted(set(conflicts)) if conflicts else 'none'}; write extra cycles: "
          f"{sorted(set(WRITE_CONFLICTS)) if WRITE_CONFLICTS else 'none'}")
    assert err < 1e-10, err


if __name__ == "__main__":
    main()

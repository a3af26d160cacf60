"""Numpy model of the L = 32 768 overlap-save segment of fir_fft32.hpp.

The 16 384-point complex transform of a segment (z[m] = x[2m] + i x[2m+1]) is
split by the parity of its bins (radix-2 decimation in frequency):

    Z[2 kappa]     = FFT_8192( z[m] + z[m + 8192] )[kappa]                 half E
    Z[2 kappa + 1] = FFT_8192( (z[m] - z[m + 8192]) W_16384^m )[kappa]     half O

Each half is the 8192-point four-step transform of fir_fft.hpp (stage 1 =
16-point DFTs across a for thread b, m = 512 a + b, twiddle W_8192^(b c);
512-point columns).  For half O the factor W_16384^m = W_32^a W_16384^b splits
into a constant per register (W_32^a, before the DFT16) and a per-thread
factor that joins the stage-1 twiddles: W_16384^(b (2c + 1)).  Bins pair
within a half (k and M - k have one parity): half E kappa <-> 8192 - kappa
(the existing lane structure, special lane included), half O kappa <->
8191 - kappa (every wave: columns w and 15 - w, task B the mirror of task A).
The inverse runs each half's 8192-point transform of conj(V) and combines

    out[m]        = out_E[m] + W_32^a out_O'[m]
    out[m + 8192] = out_E[m] - W_32^a out_O'[m]      (m = 512 a + b, a < 16)

where out_O' carries W_16384^b from its final-stage twiddles.  c[2m] =
Re out[m], c[2m+1] = -Im out[m].  The pair tables (host, long double in the
library) use the L = 32 768 spectrum of the filter at the half's bins.

Run: python scripts/fft32_model.py  (checks against numpy's convolution)
"""
import numpy as np

L = 32768
M = L // 2          # complex transform length
MH = M // 2         # per-half transform length (8192)
W = lambda n, k: np.exp(-2j * np.pi * np.asarray(k, dtype=np.float64) / n)  # noqa: E731


def stage1(z):
    """Per thread b (rows), the two halves' stage-1 column values: [16][512]."""
    zz = z.reshape(32, 512)                 # zz[a][b] = z[512 a + b]
    u = zz[:16] + zz[16:]
    d = zz[:16] - zz[16:]
    v = d * W(32, np.arange(16))[:, None]   # constants per register a
    b = np.arange(512)
    c = np.arange(16)[:, None]
    ye = np.fft.fft(u, axis=0) * W(MH, b[None, :] * c)            # W_8192^(b c)
    yo = np.fft.fft(v, axis=0) * W(M, b[None, :] * (2 * c + 1))   # W_16384^(b (2c+1))
    return ye, yo


def columns(y):
    """512-point DFT of each column c: bins kappa = c + 16 k2 -> [8192]."""
    Zc = np.fft.fft(y, axis=1)              # [c][k2]
    out = np.zeros(MH, complex)
    for c in range(16):
        out[c + 16 * np.arange(512)] = Zc[c]
    return out


def spectrum(taps, sym):
    """G = FFT_L of the filter: zero-phase (taps centred on 0) or reversed taps."""
    T = taps.size
    g = np.zeros(L)
    if sym:
        half = (T - 1) // 2
        j = np.arange(-half, half + 1)
        g[j % L] = (taps[half + j] + taps[half - j]) * 0.5
    else:
        g[:T] = taps[::-1]
    return np.fft.fft(g)


def pair_coeffs(G, k):
    """2S, 2D, W for full bins k (partner M - k), scaled 1 / (4 M) as fft_plan_build."""
    scale = 1.0 / (4 * M)
    g = G[k] * scale
    h = np.conj(G[M - k]) * scale          # L-point index M - k (k = 0: G[M])
    return 2 * (g + h), 2 * (g - h), W(L, k)


def pair_step(Zk, Zp, S2, D2, Wk):
    """fft_pair: (Z_k, Z_{M-k}) -> conj(V_k), conj(V_{M-k})."""
    P1 = S2 + D2 * Wk.imag
    Q2 = S2 - D2 * Wk.imag
    P2 = 1j * D2 * Wk.real
    Zm = np.conj(Zp)
    return np.conj(Zk * P1 + Zm * P2), Zm * Q2 - Zk * P2


def inverse_half(Vc, odd):
    """8192-point four-step transform of the half's conj(V) (bins kappa =
    c + 16 k2): columns over k2 -> b, final twiddle, DFT16 over c -> a."""
    cols = np.zeros((16, 512), complex)
    for c in range(16):
        cols[c] = np.fft.fft(Vc[c + 16 * np.arange(512)])      # index b
    b = np.arange(512)
    c = np.arange(16)[:, None]
    tw = W(M, b[None, :] * (2 * c + 1)) if odd else W(MH, b[None, :] * c)
    return np.fft.fft(cols * tw, axis=0)                        # [a][b]


def segment(x_seg, taps, sym):
    z = x_seg[0::2] + 1j * x_seg[1::2]
    ye, yo = stage1(z)
    Ze, Zo = columns(ye), columns(yo)
    Z = np.zeros(M, complex)
    Z[0::2], Z[1::2] = Ze, Zo
    assert np.allclose(Z, np.fft.fft(z), rtol=0, atol=1e-9 * np.abs(Z).max())
    G = spectrum(taps, sym)
    k = np.arange(M)
    S2, D2, Wk = pair_coeffs(G, k)
    Vc = np.zeros(M, complex)
    oP, _ = pair_step(Z, Z[(M - k) % M], S2, D2, Wk)
    Vc[:] = oP                               # conj(V_k) for every k (each pair written twice)
    oe = inverse_half(Vc[0::2], False)       # [a][b], a < 16
    oo = inverse_half(Vc[1::2], True)
    oo = oo * W(32, np.arange(16))[:, None]
    out = np.zeros(M, complex)
    out.reshape(32, 512)[:16] = oe + oo
    out.reshape(32, 512)[16:] = oe - oo
    c = np.zeros(L)
    c[0::2], c[1::2] = out.real, -out.imag
    return c


def main():
    rng = np.random.default_rng(3)
    for T, sym in [(8001, True), (4001, True), (8003, False), (30001, True)]:
        h = rng.standard_normal(T)
        if sym:
            h = (h + h[::-1]) / 2
        x = rng.standard_normal(L)
        c = segment(x, h, sym)
        half = (T - 1) // 2
        full = np.convolve(x, h[::-1])       # full[j] = sum_k h[k] x[j - (T-1) + k]
        if sym:
            # c[m] = sum_k h[k] x[m - half + k], valid m in [half, L - half)
            want = full[half + half: L - half + half][:]
            got = c[half:L - half]
            want = np.array([np.dot(h, x[m - half:m - half + T]) for m in range(half, L - half, 997)])
            got = c[half:L - half:997]
        else:
            want = np.array([np.dot(h, x[m - (T - 1):m + 1]) for m in range(T - 1, L, 997)])
            got = c[T - 1:L:997]
        err = np.abs(got - want).max() / np.abs(want).max()
        print(f"T={T} sym={sym}: max rel err {err:.2e}")
        assert err < 1e-12


if __name__ == "__main__":
    main()


# ---- emulation of the kernels' pair step on the library's own host tables ----
# tests/cpp/fft_tables_dump writes lcfir::fft_plan_tables (fir_fft.hpp) for a
# tap set; emulate() runs a segment through the transform with the pair step
# done exactly as fft_columns does it per (thread, slot): the task words'
# lane layout, the special lane's permuted bins, the general table's W base
# times W_16^i, the zero-phase table's (p1, q2) / p2 layout, c8.
PAIR_SLOTS, NT, SPECIAL_LANE = 9, 512, 35
SYM_P2 = 8 * NT


def load_tables(prefix):
    L_, halves, parts, tp, sym, reg32 = map(int, open(prefix + ".meta").read().split())
    cplx = lambda f: np.fromfile(prefix + f, np.float64).view(np.complex128)  # noqa: E731
    return {"L": L_, "halves": halves, "parts": parts, "tp": tp, "sym": bool(sym), "reg32": bool(reg32),
            "pair": cplx(".pair"), "c8": cplx(".c8"), "tw": cplx(".tw"),
            "task": np.fromfile(prefix + ".task", np.uint32)}


def _slot_col_even(s):
    return 0 if s == 0 else 8 if s == 1 else (s // 2 if s % 2 == 0 else (33 - s) // 2)


def _slot_col_odd(s):
    return (31 - s) // 2 if s & 1 else s // 2


def pair_half_emulated(Zh, table, task, h, c8, sym):
    """conj(V) of one 8192-point half from its bins Zh, as the kernel's lanes compute it."""
    out = np.full(MH, np.nan, complex)
    w16 = W(16, np.arange(8))
    col = _slot_col_even if h == 0 else _slot_col_odd
    for t in range(NT):
        tk = int(task[t])
        cA, dA, eA = col(tk & 15), (tk >> 4) & 7, (tk >> 7) & 7
        cB, dB, eB = col((tk >> 10) & 15), (tk >> 14) & 7, (tk >> 17) & 7
        special = h == 0 and t == SPECIAL_LANE
        if special:
            ks = [512 + 1024 * i if i < 4 else 1024 * (i - 4) for i in range(8)]
            pairs = [(k, (MH - k) % MH) for k in ks]
        else:
            pairs = [(cA + 16 * (dA + 8 * eA + 64 * i), cB + 16 * (dB + 8 * eB + 64 * (7 - i))) for i in range(8)]
        for i, (kp, kq) in enumerate(pairs):
            P, Q = Zh[kp], Zh[kq]
            o = i * NT + t
            if sym:
                p1, q2 = table[o].real, table[o].imag
                p2v = table[SYM_P2 + (i >> 1) * NT + t]
                p2 = p2v.imag if i & 1 else p2v.real
                oP = np.conj(P * p1 + np.conj(Q) * 1j * p2)
                oQ = np.conj(Q) * q2 - P * 1j * p2
            else:
                S2, D2 = table[o], table[PAIR_SLOTS * NT + o]
                wb = 1j if (special and i >= 4) else table[2 * PAIR_SLOTS * NT + t]
                Wk = wb * w16[i]
                P1, Q2, P2 = S2 + D2 * Wk.imag, S2 - D2 * Wk.imag, 1j * D2 * Wk.real
                Zm = np.conj(Q)
                oP, oQ = np.conj(P * P1 + Zm * P2), Zm * Q2 - P * P2
            out[kp], out[kq] = oP, oQ
        if special:
            out[MH // 2] = np.conj(Zh[MH // 2] * c8)
    assert not np.isnan(out).any()
    return out


def emulate(x_seg, tb, part=0):
    """c[0, L) of one segment through the library's tables (partition `part`)."""
    table_n = 3 * PAIR_SLOTS * NT
    if tb["halves"] == 1:
        z = x_seg[0::2] + 1j * x_seg[1::2]
        Vc = pair_half_emulated(np.fft.fft(z), tb["pair"][part * table_n:(part + 1) * table_n], tb["task"], 0,
                                tb["c8"][part], tb["sym"])
        out = np.fft.fft(Vc)
    else:
        z = x_seg[0::2] + 1j * x_seg[1::2]
        Z = np.fft.fft(z)
        base = 2 * part * table_n
        Ve = pair_half_emulated(Z[0::2], tb["pair"][base:base + table_n], tb["task"][:NT], 0, tb["c8"][part],
                                tb["sym"])
        Vo = pair_half_emulated(Z[1::2], tb["pair"][base + table_n:base + 2 * table_n], tb["task"][NT:], 1, 0,
                                tb["sym"])
        oe = inverse_half(Ve, False)
        oo = inverse_half(Vo, True) * W(32, np.arange(16))[:, None]
        out = np.zeros(M, complex)
        out.reshape(32, 512)[:16] = oe + oo
        out.reshape(32, 512)[16:] = oe - oo
    c = np.zeros(2 * out.size)
    c[0::2], c[1::2] = out.real, -out.imag
    return c

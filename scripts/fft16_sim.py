"""Index-flow and LDS-bank check of the 16-wave FFT kernel (csrc/fir_fft16.hpp).

1024 threads: wave w (0..15) owns column c = w of the 16 x 512 four-step
decomposition of the M = 8192-point complex FFT; thread t = 64 w + L with
h = L >> 5 and b = 32 w + (L & 31) shares the 16-point DFTs of stage 1 and
of the final phase with its partner lane L ^ 32 (one v_permlane32_swap per
dword).  The column stages are the 8-wave kernel's (fir_fft.hpp; their
layouts are checked by scripts/fft_lds_sim.py).  The pair step is split:
each lane computes conj(V_k) for its own bins from its own Z_k and the
partner column's Z_{M-k}, read from LDS after one workgroup barrier.

Simulated here with numpy (complex128), lane by lane and register by
register, before any GPU time is spent:
  * stage 1 -> columns -> pair step -> inverse columns -> final phase
    reproduces the real overlap-save convolution of the kernel's contract;
  * every thread writes in stage 1 exactly the LDS addresses it read in
    the previous unit's final phase (no barrier between the two);
  * the new LDS accesses (stage-1 writes, C-output writes, partner reads,
    final reads) are bank-conflict free under the gfx950 lane-group rules.

usage: python scripts/fft16_sim.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fft_lds_sim as v3  # noqa: E402  (lane groups, fx layouts)

M = 8192
L_REAL = 2 * M
W = v3.W
dft = v3.dft


def blk(c, p):
    """LDS block of column c at the start of a unit of parity p (at its end,
    after the pair step moved it to the partner's block, blk(c, 1 - p))."""
    return c if p == 0 else (16 - c) % 16


def swap32(regs, i, j):
    """v_permlane32_swap(vdst = reg i, vsrc = reg j) on a [64][R] register
    file: lanes 32..63 of reg i trade places with lanes 0..31 of reg j."""
    hi = regs[32:, i].copy()
    regs[32:, i] = regs[:32, j]
    regs[:32, j] = hi


def pair_coeffs(G):
    """Per-bin (a, b) of the zero-phase pair step: conj(V_k) = conj(Z_k) a_k +
    Z_{M-k} (-i b_k), from the real spectrum G (length L) of the centred taps,
    scaled like fft_plan_build (1 / 4M)."""
    a = np.zeros(M)
    b = np.zeros(M)
    for k in range(M):
        g0 = G[k] / (4 * M)
        g1 = G[M - k] / (4 * M)
        s2, d2 = 2 * (g0 + g1), 2 * (g0 - g1)
        wl = W(L_REAL, k)
        a[k] = s2 + d2 * wl.imag
        b[k] = d2 * wl.real
    return a, b


def unit(z, coef, p, lds):
    """One unit of the kernel on the packed samples z (M complex); lds holds
    the 16 x 512 work array (in/out).  Returns v (conj-trick output, M
    complex) and the address sets of stage 1 and the final phase per thread."""
    a_tab, b_tab = coef
    wrote1, read_final = {}, {}
    # ---- stage 1
    for w in range(16):
        R = np.zeros((64, 8), complex)
        for Ln in range(64):
            h, b = Ln >> 5, 32 * w + (Ln & 31)
            R[Ln] = dft(np.array([z[512 * (2 * a + h) + b] for a in range(8)]))
        for i in range(4):
            swap32(R, i, 4 + i)
        for Ln in range(64):
            h, b = Ln >> 5, 32 * w + (Ln & 31)
            addr = set()
            for i in range(4):
                o = R[Ln, 4 + i] * W(16, i + 4 * h)
                y0, y1 = R[Ln, i] + o, R[Ln, i] - o
                for c, y in ((4 * h + i, y0), (8 + 4 * h + i, y1)):
                    lds[blk(c, p), b] = y * W(M, b * c)
                    addr.add((blk(c, p), b))
            wrote1[(w, Ln)] = addr
    # ---- forward column DFTs (fft_lds_sim semantics) -> C output at 64 e2 + L
    Xc = np.zeros((16, 512), complex)  # [c][r], k = c + 16 r
    for c in range(16):
        Xc[c] = dft(lds[blk(c, p)])  # = the column DFT; bins r = L + 64 e2
    for c in range(16):
        lds[blk(c, p)] = Xc[c]  # C output, linear position r
    # ---- pair step (each lane: own bins + the partner column's mirror)
    V = np.zeros((16, 512), complex)
    for c in range(16):
        cb = (16 - c) % 16
        for Ln in range(64):
            for e2 in range(8):
                r = Ln + 64 * e2
                pos = (512 - r) % 512 if c == 0 else 511 - r
                q = lds[blk(cb, p), pos]
                own = Xc[c, r]
                k = c + 16 * r
                assert (cb + 16 * pos) % M == (M - k) % M
                V[c, r] = np.conj(own) * a_tab[k] + q * (-1j * b_tab[k])
    # ---- inverse column DFTs (forward-signed, conj trick) into blk(c, 1 - p)
    for c in range(16):
        lds[blk(c, 1 - p)] = dft(V[c])  # U[c][b] before the W8192^(bc) twiddle
    # ---- final phase
    v = np.zeros(M, complex)
    for w in range(16):
        R = np.zeros((64, 8), complex)
        for Ln in range(64):
            h, b = Ln >> 5, 32 * w + (Ln & 31)
            addr = set()
            for i in range(4):
                cf, cg = 4 * h + i, 8 + 4 * h + i
                f = lds[blk(cf, 1 - p), b] * W(M, b * cf)
                g = lds[blk(cg, 1 - p), b] * W(M, b * cg)
                addr |= {(blk(cf, 1 - p), b), (blk(cg, 1 - p), b)}
                R[Ln, i], R[Ln, 4 + i] = f + g, f - g
            read_final[(w, Ln)] = addr
        for i in range(4):
            swap32(R, i, 4 + i)
        for Ln in range(64):
            h, b = Ln >> 5, 32 * w + (Ln & 31)
            r = R[Ln] * (W(16, np.arange(8)) if h else 1.0)
            out = dft(r)
            for a in range(8):
                v[512 * (2 * a + h) + b] = out[a]
    return v, wrote1, read_final


def check_flow(seed=3, ntaps=401):
    """Zero-phase overlap-save of one unit against a direct convolution."""
    rng = np.random.default_rng(seed)
    half = (ntaps - 1) // 2
    hh = rng.standard_normal(half + 1)
    taps = np.concatenate([hh[:0:-1], hh])  # symmetric, length ntaps
    g = np.zeros(L_REAL)
    for j in range(-half, half + 1):
        g[j % L_REAL] = taps[half + j]
    G = np.fft.fft(g).real
    coef = pair_coeffs(G)
    xs = rng.standard_normal(L_REAL)
    z = xs[0::2] + 1j * xs[1::2]
    lds = np.zeros((16, 512), complex)
    errs = []
    for p in (0, 1):
        v, wrote1, read_final = unit(z, coef, p, lds)
        c_out = np.empty(L_REAL)
        c_out[0::2] = v.real
        c_out[1::2] = -v.imag
        ref = np.array([sum(taps[half + j] * xs[(m - j) % L_REAL] for j in range(-half, half + 1))
                        for m in range(half, L_REAL - half, 97)])
        got = c_out[half:L_REAL - half:97]
        errs.append(np.max(np.abs(got - ref)) / np.max(np.abs(ref)))
        # the next unit (parity 1 - p) writes in stage 1 what this one read last
        _, wrote_next, _ = unit(z, coef, 1 - p, lds.copy())
        assert all(wrote_next[t] == read_final[t] for t in read_final), "stage-1 / final address sets"
    return max(errs)


def check_banks():
    rep = {}
    # stage-1 writes / final reads: lane -> index b inside the block
    idx = [32 * 0 + (Ln & 31) for Ln in range(64)]
    rep["stage-1 write"] = v3.conflicts_write(idx)
    rep["final read"] = v3.conflicts_read(idx)
    # C output: position 64 e2 + L; partner read: 511 - r (c != 0), (512 - r) % 512 (c = 0)
    rep["C-output write"] = sum(v3.conflicts_write([64 * e2 + Ln for Ln in range(64)]) for e2 in range(8))
    rep["partner read"] = sum(v3.conflicts_read([511 - Ln - 64 * e2 for Ln in range(64)]) for e2 in range(8))
    rep["partner read c0"] = sum(v3.conflicts_read([(512 - Ln - 64 * e2) % 512 for Ln in range(64)])
                                 for e2 in range(8))
    # column stages with the task (d1, e1) = (L & 7, L >> 3) of every wave
    r = 0
    for l1 in range(8):
        r += v3.conflicts_read([v3.x2(l1, Ln & 7, Ln >> 3) for Ln in range(64)])
    rep["x2 read"] = r
    rep["x3 write"] = sum(v3.conflicts_write([v3.x3(Ln & 7, Ln >> 3, b0) for Ln in range(64)]) for b0 in range(8))
    return rep


def main():
    rep = check_banks()
    for k, v in rep.items():
        print(f"{k:24s} extra cycles {v}")
    assert all(v == 0 for v in rep.values()), "bank conflicts"
    err = check_flow()
    print("overlap-save flow rel err", err)
    assert err < 1e-12


if __name__ == "__main__":
    main()

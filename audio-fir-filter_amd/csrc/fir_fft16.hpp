// fir_fft16.hpp -- the f64 overlap-save FFT kernel at four waves per SIMD.
//
// Same contract, segment geometry and zero-phase form as fir_fft.hpp's
// kFftOutSym kernel (L = 16384 real samples per unit, one complex M = 8192
// FFT of the packed even/odd samples, B = L - T + 1 outputs), reorganised
// for 1 024 threads: 16 waves per workgroup, one workgroup (137 KiB of LDS)
// per CU, so every SIMD holds FOUR waves instead of two.
//
// Why: the 8-wave kernel is bound by f64 VALU issue at two waves per SIMD.
// Issue is arbitrated oldest-first, so the younger wave of each SIMD gets
// the leftover slots, runs alone at the single-wave rate (half the pipe)
// once its partner waits at a barrier, and the SIMD idles half its f64
// pipe for about a third of every segment.  With four waves
// per SIMD two of them keep the pipe full while the others wait on LDS or
// at a barrier.
//
// Decomposition, M = 16 x 512 as before; thread t = 64 w + L, h = L >> 5,
// b = 32 w + (L & 31):
//   stage 1   the 16-point DFT over z[512 a + b] is shared by lanes L and
//             L ^ 32: each does the 8-point DFT over a = 2 a' + h, one
//             v_permlane32_swap per dword trades halves, and the radix-2
//             butterfly gives lower lanes columns {0..3, 8..11}, upper
//             lanes {4..7, 12..15}; times W_8192^(b c) into LDS.
//   columns   wave w owns column c = w: the 8 x 8 x 8 column DFT with the
//             8-wave kernel's wave-local exchanges (fx1, fx2 layouts).
//   pair      the bins k and M - k sit in columns c and 16 - c, i.e. in two
//             waves.  Each wave writes its column's bins to LDS, one
//             workgroup barrier, then every lane reads the partner column's
//             mirror bins and computes conj(V_k) for its OWN bins only:
//                 conj(V_k) = conj(Z_k) a_k + Z_{M-k} (-i b_k)
//             with (a_k, b_k) per bin from the host (long double) -- the
//             8-wave kernel's P-role formula, which holds for every bin,
//             including the self-paired 0 and M/2.
//   inverse   each wave continues in its partner's block (it has just read
//             it; the partner reads this wave's block), so no second
//             barrier guards the reuse; columns move block c <-> 16 - c
//             every unit (fft16_blk, parity of the unit).
//   final     the 16-point DFTs over the columns, split over the lane pair
//             like stage 1 (DIF: even outputs in lower lanes, odd in upper).
// Per unit: 3 workgroup barriers, 7 LDS round trips of the 128 KiB array.
// Index flow, address sets and bank patterns: scripts/fft16_sim.py.
#pragma once

#include "fir_fft.hpp"

namespace lcfir {

constexpr int kFft16NT = 1024;
// pair table of the 16-wave kernel: double2 (a, b) per (slot e2, thread t)
constexpr size_t kFft16PairTable = (size_t)8 * kFft16NT;

// LDS block of column c in a unit of parity p (p = rnd & 1): a column's
// inverse data ends in its partner's block, blk(c, p ^ 1)
__host__ __device__ __forceinline__ int fft16_blk(int c, int p) { return p ? (16 - c) & 15 : c; }

// v_permlane32_swap on a double2 pair: lanes 32..63 of a trade with lanes
// 0..31 of b (four dwords)
__device__ __forceinline__ void fft16_swap(double2 &a, double2 &b) {
    const uint64_t ax = __builtin_bit_cast(uint64_t, a.x), ay = __builtin_bit_cast(uint64_t, a.y);
    const uint64_t bx = __builtin_bit_cast(uint64_t, b.x), by = __builtin_bit_cast(uint64_t, b.y);
    const auto r0 = __builtin_amdgcn_permlane32_swap((unsigned)ax, (unsigned)bx, false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap((unsigned)(ax >> 32), (unsigned)(bx >> 32), false, false);
    const auto r2 = __builtin_amdgcn_permlane32_swap((unsigned)ay, (unsigned)by, false, false);
    const auto r3 = __builtin_amdgcn_permlane32_swap((unsigned)(ay >> 32), (unsigned)(by >> 32), false, false);
    a.x = __builtin_bit_cast(double, (uint64_t)r0[0] | (uint64_t)r1[0] << 32);
    b.x = __builtin_bit_cast(double, (uint64_t)r0[1] | (uint64_t)r1[1] << 32);
    a.y = __builtin_bit_cast(double, (uint64_t)r2[0] | (uint64_t)r3[0] << 32);
    b.y = __builtin_bit_cast(double, (uint64_t)r2[1] | (uint64_t)r3[1] << 32);
}

// W_16^(i + 4h), i = 0..3: the radix-2 twiddle of the lane pair's butterfly
__device__ __forceinline__ double2 fft16_half_tw(int i, bool hi) {
    switch (i) {
    case 0: return hi ? make_double2(0.0, -1.0) : make_double2(1.0, 0.0);
    case 1: return hi ? make_double2(-kS1, -kC1) : make_double2(kC1, -kS1);
    case 2: return hi ? make_double2(-kR2, -kR2) : make_double2(kR2, -kR2);
    default: return hi ? make_double2(-kC1, -kS1) : make_double2(kS1, -kC1);
    }
}

// t[j] = W_8192^(b c_j) for the lane's columns c_j = 4h + j (j < 4),
// 8 + 4h + j - 4 (j >= 4), from w1 = W_8192^b (depth <= 5 products)
__device__ __forceinline__ void fft16_col_tw(double2 w1, bool hi, double2 (&t)[8]) {
    const double2 w2 = cmul(w1, w1), w3 = cmul(w2, w1), w4 = cmul(w2, w2), w8 = cmul(w4, w4);
    const double2 base = make_double2(hi ? w4.x : 1.0, hi ? w4.y : 0.0);
    t[0] = base;
    t[1] = cmul(base, w1);
    t[2] = cmul(base, w2);
    t[3] = cmul(base, w3);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[4 + j] = cmul(t[j], w8);
}

// Samples of one unit for thread (b, h): v[a] = (x_seg[2m], x_seg[2m+1]),
// m = 512 (2a + h) + b -- fft_load_unit's range-checked buffer loads with
// the lane pair's stride (m0 = 512 h + b, step 1024).
__device__ __forceinline__ void fft16_load_unit(const DirectParams &p, int ch, int64_t n0, int m0,
                                                float2 (&v)[8]) {
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(x), (short)0, (int)((p.x_hi - p.x_lo) * 4), 0x00020000);
    const int64_t w0 = n0 - p.half - p.x_lo;
    const int off0 = (int)(w0 * 4) + 8 * m0; // may be negative: wraps out of range, reads 0
    // One code path for interior and edge units (two paths, merged, cost
    // ~70 VGPR spills at 128 VGPRs): every sample is its own range-checked
    // dword load, and the odd samples carry the sc0 policy bit so the two
    // halves of a pair are never merged into one dwordx2, whose all-or-
    // nothing range check would drop the in-range half of a pair that
    // straddles the window's edge.
#pragma unroll
    for (int a = 0; a < 8; ++a) {
        const int off = off0 + 8 * 1024 * a;
        v[a].x = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
        v[a].y = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, 1));
    }
}

__device__ __forceinline__ void fft16_peak_stage(float *pk_lds, float pk) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) pk = fmaxf(pk, __shfl_xor(pk, s, 64));
    if ((threadIdx.x & 63) == 0) pk_lds[threadIdx.x >> 6] = pk;
}
__device__ __forceinline__ void fft16_peak_commit(const DirectParams &p, int ch, const float *pk_lds) {
    float pk = pk_lds[0];
#pragma unroll
    for (int w = 1; w < kFft16NT / 64; ++w) pk = fmaxf(pk, pk_lds[w]);
    atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(pk));
}

// threadIdx.x behind an empty asm: every phase re-derives its lane values
// from its own copy, so the compiler cannot share them across the unit's
// barriers (shared, they stay live through the column stages and spill at
// four waves per SIMD, 128 VGPRs)
__device__ __forceinline__ int fft16_tid() {
    int j = threadIdx.x;
    asm volatile("" : "+v"(j));
    return j;
}

// Persistent: one 1024-thread workgroup per CU walks units fft_unit(rnd, ...)
// of the nch x nseg (channel, segment) grid; zero-phase form only
// (fft_plan_build's sym tables; outputs c in [half, L - half)).  A template
// (kOut = kFftOutSym only) so that host-only builds of the header emit nothing.
template <int kOut>
__global__ __launch_bounds__(kFft16NT) void fir_fft16_f64_kernel(DirectParams p, const double2 *__restrict__ pair,
                                                                const double2 *__restrict__ tw, int B,
                                                                FftGrid gd) {
    extern __shared__ double2 flds[];
    double2 *twl = flds + kFftM; // kFftTw twiddles, LDS-resident
    for (int i = threadIdx.x; i < kFftTw; i += kFft16NT) twl[i] = tw[i];
    const int m0 = (int)((threadIdx.x & 32) << 4) + (int)(((threadIdx.x >> 6) << 5) | (threadIdx.x & 31)); // 512 h + b
    float2 v[8];
    {
        const int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units);
        const int c0 = fft_div(u, gd);
        fft16_load_unit(p, c0, p.seg0 + (int64_t)(u - c0 * gd.nseg) * B, m0, v);
    }
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    float pk_run = 0.0f;
    int pk_ch = -1;
    float *pk_lds = reinterpret_cast<float *>(twl + kFftTw);
    int pk_pending = -1;
    int rnd = 0;
    for (int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units); u < gd.units;
         u = fft_unit32(++rnd, blockIdx.x, gridDim.x, gd.units)) {
    const int par = (int)(rnd & 1);
    const int ch = fft_div(u, gd);
    const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;

    // ---- stage 1: lane pair (b, h): 8-point DFT over a' -> swap -> radix-2
    {
        const int j = fft16_tid(), lane = j & 63, hh = lane >> 5, b = ((j >> 6) << 5) | (lane & 31);
        const bool hi = hh != 0;
        double2 s[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) s[a] = make_double2((double)v[a].x, (double)v[a].y);
        dft8(s); // lower: E[c'], upper: O[c']
        double2 wt[8];
        fft16_col_tw(twl[b], hi, wt);
#pragma unroll
        for (int i = 0; i < 4; ++i) fft16_swap(s[i], s[4 + i]);
        // lower: s[i] = E[i], s[4+i] = O[i]; upper: s[i] = E[4+i], s[4+i] = O[4+i]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double2 o = cmul(s[4 + i], fft16_half_tw(i, hi));
            const double2 y0 = cadd(s[i], o), y1 = csub(s[i], o);
            const int c0 = 4 * hh + i, c1 = 8 + 4 * hh + i;
            // no barrier before these writes: thread j rewrites exactly the
            // addresses it read in the previous unit's final phase
            flds[512 * fft16_blk(c0, par) + b] = cmul(y0, wt[i]);
            flds[512 * fft16_blk(c1, par) + b] = cmul(y1, wt[4 + i]);
        }
        __syncthreads(); // B1
        if (pk_pending >= 0) {
            if (threadIdx.x == 0) fft16_peak_commit(p, pk_pending, pk_lds);
            pk_pending = -1;
        }
    }

    // ---- column c = w in block fft16_blk(w, par): stages A, B, C (fir_fft.hpp layouts)
    const int j = fft16_tid(), lane = j & 63, w = j >> 6;
    double2 x[8], tws[8];
    double2 *blk0 = flds + 512 * fft16_blk(w, par);
    const int l1 = lane & 7, d1s = lane >> 3;
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = blk0[lane + 64 * t];
    powers8(twl[512 + lane], tws);
    dft8(x);
    twiddle8(x, tws);
#pragma unroll
    for (int d1 = 0; d1 < 8; ++d1) blk0[fx1(lane, d1)] = x[d1];
    wave_lds_sync();
#pragma unroll
    for (int l2 = 0; l2 < 8; ++l2) x[l2] = blk0[fx1(l1 + 8 * l2, d1s)];
    powers8(twl[512 + 8 * l1], tws);
    dft8(x);
    twiddle8(x, tws);
#pragma unroll
    for (int e1 = 0; e1 < 8; ++e1) blk0[fx2(l1, d1s, e1)] = x[e1];
    wave_lds_sync();
    // stage C: task (d1, e1) = (lane & 7, lane >> 3) -> bins k = w + 16 (lane + 64 e2)
#pragma unroll
    for (int l = 0; l < 8; ++l) x[l] = blk0[fx2(l, l1, d1s)];
    dft8(x);
    // C output at linear position r = lane + 64 e2 of the column's block
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) blk0[lane + 64 * e2] = x[e2];
    __syncthreads(); // B2

    // ---- pair step: own Z_k (registers) + the partner column's Z_{M-k} (LDS)
    const int cb = (16 - w) & 15;
    double2 *blkp = flds + 512 * fft16_blk(cb, par); // = block fft16_blk(w, par ^ 1)
    {
        const int pos0 = (w == 0 ? 512 : 511) - lane; // mirror of r = lane: 511 - r (512 - r for column 0)
        double2 q[8], ab[8];
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) ab[e2] = pair[kFft16NT * e2 + j];
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) q[e2] = blkp[(pos0 - 64 * e2) & 511];
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) {
            const double a = ab[e2].x, bb = ab[e2].y;
            x[e2] = make_double2(__builtin_fma(a, x[e2].x, bb * q[e2].y), -__builtin_fma(a, x[e2].y, bb * q[e2].x));
        }
    }
    // ---- prefetch the next unit's samples (unconditional: the last unit reloads itself);
    // pinned behind the pair step, whose operands would otherwise share the registers
    __builtin_amdgcn_sched_barrier(0);
    {
        const int un1 = fft_unit32(rnd + 1, blockIdx.x, gridDim.x, gd.units);
        const int un = un1 < gd.units ? un1 : u;
        const int cn = fft_div(un, gd);
        fft16_load_unit(p, cn, p.seg0 + (int64_t)(un - cn * gd.nseg) * B, m0, v);
    }
    // ---- inverse stage A' (task d' = lane): radix-8 over e2 -> beta0; * W_512^(beta0 lane)
    // in the partner's block: this wave has read it, and only this wave reads it
    powers8(twl[512 + lane], tws);
    dft8(x);
    twiddle8(x, tws);
#pragma unroll
    for (int b0 = 0; b0 < 8; ++b0) blkp[fx3(l1, d1s, b0)] = x[b0];
    wave_lds_sync();
    // ---- stage B': lane (d1, beta0) gathers e1; radix-8 -> gamma0; * W_64^(gamma0 d1)
#pragma unroll
    for (int e1 = 0; e1 < 8; ++e1) x[e1] = blkp[fx3(l1, e1, d1s)];
    powers8(twl[512 + 8 * l1], tws);
    dft8(x);
    twiddle8(x, tws);
#pragma unroll
    for (int g0 = 0; g0 < 8; ++g0) blkp[fx4(l1, d1s, g0)] = x[g0];
    wave_lds_sync();
    // ---- stage C': lane rho = beta0 + 8 gamma0 gathers d1; radix-8 -> gamma1
#pragma unroll
    for (int dd = 0; dd < 8; ++dd) x[dd] = blkp[fx4(dd, l1, d1s)];
    dft8(x);
#pragma unroll
    for (int g1 = 0; g1 < 8; ++g1) blkp[lane + 64 * g1] = x[g1]; // b = lane + 64 gamma1
    __syncthreads(); // B3

    // ---- final: lane pair (b, h): * W_8192^(b c), radix-2 (DIF), swap, 8-point DFT
    const int jf = fft16_tid(), hh = (jf >> 5) & 1, b = ((jf >> 6) << 5) | (jf & 31);
    const bool hi = hh != 0;
    double2 r[8], wt[8];
    fft16_col_tw(twl[b], hi, wt);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double2 f = cmul(flds[512 * fft16_blk(4 * hh + i, par ^ 1) + b], wt[i]);
        const double2 g = cmul(flds[512 * fft16_blk(8 + 4 * hh + i, par ^ 1) + b], wt[4 + i]);
        r[i] = cadd(f, g);
        r[4 + i] = cmul(csub(f, g), fft16_half_tw(i, hi));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) fft16_swap(r[i], r[4 + i]);
    dft8(r); // lower: out[2a''], upper: out[2a''+1] -> v[512 (2a'' + h) + b]

    // ---- outputs: c[2m] = Re, c[2m+1] = -Im, m = 512 (2a + h) + b, valid c in [half, L - half)
    __builtin_amdgcn_s_waitcnt(kVmcnt0); // the prefetch has landed long ago
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
        yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
    const int cmin = p.half, cmax = kFftL - p.half;
    const int64_t off = n0 - cmin - p.start;
    const int64_t oend = p.end - p.start;
    float pk = 0.0f;
    if (n0 >= p.start && n0 + B <= p.end) {
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const int c = 2 * (512 * (2 * a + hh) + b);
            const float f0 = (float)r[a].x, f1 = (float)(-r[a].y);
            const bool ok = c >= cmin && c < cmax;
            const int ob = ok ? (int)((off + c) * 4) : (int)0x80000000;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ob, 0, kNtStore);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ob + 4, 0, kNtStore);
            pk = fmaxf(pk, ok ? fmaxf(fabsf(f0), fabsf(f1)) : 0.0f);
        }
    } else {
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const int c = 2 * (512 * (2 * a + hh) + b);
            const float f0 = (float)r[a].x, f1 = (float)(-r[a].y);
            const int64_t o = off + c;
            const bool ok0 = c >= cmin && c < cmax && o >= 0 && o < oend,
                       ok1 = c + 1 >= cmin && c + 1 < cmax && o + 1 >= 0 && o + 1 < oend;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(o * 4) : (int)0x80000000, 0,
                                                  kNtStore);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ok1 ? (int)(o * 4 + 4) : (int)0x80000000,
                                                  0, kNtStore);
            pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
        }
    }
    if (ch != pk_ch) {
        if (p.peak && pk_ch >= 0) {
            fft16_peak_stage(pk_lds, pk_run);
            pk_pending = pk_ch;
            asm volatile("" : "+v"(pk_pending));
        }
        pk_run = 0.0f;
        pk_ch = ch;
    }
    pk_run = fmaxf(pk_run, pk);
    }
    if (p.peak && pk_ch >= 0) {
        __syncthreads();
        if (pk_pending >= 0 && threadIdx.x == 0) fft16_peak_commit(p, pk_pending, pk_lds);
        __syncthreads();
        fft16_peak_stage(pk_lds, pk_run);
        __syncthreads();
        if (threadIdx.x == 0) fft16_peak_commit(p, pk_ch, pk_lds);
    }
}

// work array + twiddles + one f32 peak slot per wave
constexpr size_t fft16_lds_bytes() { return sizeof(double2) * (size_t)(kFftM + kFftTw) + 4 * (kFft16NT / 64); }

} // namespace lcfir

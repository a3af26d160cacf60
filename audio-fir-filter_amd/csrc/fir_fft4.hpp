// fir_fft4.hpp -- the f64 overlap-save FFT kernel at ONE wave per SIMD.
//
// fir_fft.hpp's algorithm, tables and LDS layouts unchanged, on 256 threads
// (4 waves, one per SIMD, up to 512 VGPRs each) instead of 512: thread t
// does the work of the 8-wave kernel's threads t and t + 256 ("halves"
// h = 0, 1), so wave v owns the column pairs of the 8-wave kernel's waves v
// and v + 4 -- four columns -- and software-pipelines all four through every
// wave-local LDS exchange.
//
// Why: the 8-wave kernel keeps the f64 pipe only
// ~55 % busy although one wave alone can drive it at ~87 % with this
// arithmetic (tools/valu_mix.hip).  The time goes to the chain of LDS round
// trips, which the two waves of a SIMD reach in near lockstep.  Here one
// wave covers each column's exchange with three other columns' arithmetic
// instead of one, and there is no second wave on the SIMD to compete for
// issue; the register file holds both halves' state.
#pragma once

#include "fir_fft.hpp"

namespace lcfir {

constexpr int kFft4NT = 256;

__device__ __forceinline__ void fft4_peak_stage(float *pk_lds, float pk) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) pk = fmaxf(pk, __shfl_xor(pk, s, 64));
    if ((threadIdx.x & 63) == 0) pk_lds[threadIdx.x >> 6] = pk;
}
__device__ __forceinline__ void fft4_peak_commit(const DirectParams &p, int ch, const float *pk_lds) {
    float pk = pk_lds[0];
#pragma unroll
    for (int w = 1; w < kFft4NT / 64; ++w) pk = fmaxf(pk, pk_lds[w]);
    atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(pk));
}

// Outputs of one half (fir_fft_f64_kernel's output section for thread j):
// c[2m] = Re a[r], c[2m+1] = -Im a[r], m = 512 r + j.  Returns max |y| stored.
template <int kOut>
__device__ __forceinline__ float fft4_store(const DirectParams &p, const double2 (&a)[16], int j, int ch,
                                            int64_t n0, int B) {
    constexpr bool kSym = kOut == kFftOutSym;
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
        yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
    const int cmin = kSym ? p.half : p.ntaps - 1;
    const int cmax = kSym ? kFftL - p.half : kFftL;
    const int64_t off = n0 - cmin - p.start;
    const int64_t oend = p.end - p.start;
    float pk = 0.0f;
    if constexpr (kOut == kFftOutF32 || kSym) {
        if (n0 >= p.start && n0 + B <= p.end) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int c = 2 * (j + 512 * r);
                const float f0 = (float)a[r].x, f1 = (float)(-a[r].y);
                const bool ok = c >= cmin && (!kSym || c < cmax);
                const int ob = ok ? (int)((off + c) * 4) : (int)0x80000000;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ob, 0, kNtStore);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ob + 4, 0, kNtStore);
                pk = fmaxf(pk, ok ? fmaxf(fabsf(f0), fabsf(f1)) : 0.0f);
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int c = 2 * (j + 512 * r);
                const float f0 = (float)a[r].x, f1 = (float)(-a[r].y);
                const int64_t o = off + c;
                const bool ok0 = c >= cmin && c < cmax && o >= 0 && o < oend,
                           ok1 = c + 1 >= cmin && c + 1 < cmax && o + 1 >= 0 && o + 1 < oend;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(o * 4) : (int)0x80000000, 0,
                                                      kNtStore);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                      ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, kNtStore);
                pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
            }
        }
    } else {
        double *zb = p.y64 + (int64_t)ch * p.y64_stride;
        const __amdgpu_buffer_rsrc_t zs = __builtin_amdgcn_make_buffer_rsrc(zb, (short)0, (int)(oend * 8), 0x00020000);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 2 * (j + 512 * r);
            const int64_t o = off + c;
            const bool ok0 = c >= cmin && o >= 0 && o < oend, ok1 = c + 1 >= cmin && o + 1 >= 0 && o + 1 < oend;
            const int oz0 = ok0 ? (int)(o * 8) : (int)0x80000000;
            const int oz1 = ok1 ? (int)(o * 8 + 8) : (int)0x80000000;
            double v0 = a[r].x, v1 = -a[r].y;
            if constexpr (kOut != kFftOutFirst) {
                v0 += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zs, oz0, 0, 0));
                v1 += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zs, oz1, 0, 0));
            }
            if constexpr (kOut == kFftOutLast) {
                const float f0 = (float)v0, f1 = (float)v1;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(o * 4) : (int)0x80000000, 0,
                                                      kNtStore);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                      ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, kNtStore);
                pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
            } else {
                using b64_t = decltype(__builtin_amdgcn_raw_buffer_load_b64(zs, 0, 0, 0));
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(b64_t, v0), zs, oz0, 0, kNtStore);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(b64_t, v1), zs, oz1, 0, kNtStore);
            }
        }
    }
    return pk;
}

// Pair-table registers of one half: the real p1, q2, p2 per slot in zero-phase
// form, complex 2S and 2D otherwise, plus the W_L^k base of slot 0.
template <int kOut>
struct Fft4Pair {
    static constexpr bool kSym = kOut == kFftOutSym;
    double2 qs[kSym ? 1 : 8], qd[kSym ? 1 : 8];
    double2 qpq[kSym ? 8 : 1], qp2[kSym ? 4 : 1]; // zero-phase: (p1, q2) per slot, p2 of slots 2m, 2m+1
    double2 wbase;
};

// the 8-wave kernel's pair-table loads for its thread j (issued ahead of stage
// C: L2 latency off the path)
template <int kOut>
__device__ __forceinline__ void fft4_pair_load(Fft4Pair<kOut> &q, const double2 *__restrict__ pair, int j) {
    if constexpr (Fft4Pair<kOut>::kSym) {
        const double2 *t = pair + j;
#pragma unroll
        for (int i = 0; i < 8; ++i) q.qpq[i] = t[kFftSymPQ + 512 * i];
#pragma unroll
        for (int m = 0; m < 4; ++m) q.qp2[m] = t[kFftSymP2 + 512 * m];
    } else {
        const double2 *t = pair + j;
        q.wbase = pair[2 * kFftPairSlots * 512 + j];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            q.qs[i] = t[512 * i];
            q.qd[i] = t[kFftPairSlots * 512 + 512 * i];
        }
    }
}

// The pair step of one half (fir_fft_f64_kernel's, for the 8-wave thread of
// wave w): pairs (x0[i], x1[7-i]); wave 0's special lane permuted first.
template <int kOut>
__device__ __forceinline__ void fft4_pair(double2 (&x0)[8], double2 (&x1)[8], const Fft4Pair<kOut> &q, int w,
                                          int lane, double2 c8) {
    const bool w0 = __builtin_amdgcn_readfirstlane(w) == 0; // a scalar, wave-uniform branch
    const bool sp = w0 && lane == kFftSpecialLane;
    double2 wb_hi = q.wbase;
    double2 v4 = x1[4];
    if (w0) {
        v4 = cconj(cmul(v4, c8));
        if constexpr (!Fft4Pair<kOut>::kSym) wb_hi = csel(sp, make_double2(0.0, 1.0), q.wbase);
        fft_w0_permute_in(x0, x1, sp);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if constexpr (Fft4Pair<kOut>::kSym)
            fft_pair_sym(x0[i], x1[7 - i], q.qpq[i].x, q.qpq[i].y, (i & 1) ? q.qp2[i >> 1].y : q.qp2[i >> 1].x,
                         x0[i], x1[7 - i]);
        else
            fft_pair(x0[i], x1[7 - i], fft_pair_w(i < 4 ? q.wbase : wb_hi, i), q.qs[i], q.qd[i], x0[i], x1[7 - i]);
    }
    if (w0) fft_w0_permute_out(x0, x1, sp, v4);
}

template <int kOut>
__global__ __launch_bounds__(kFft4NT) void fir_fft4_f64_kernel(DirectParams p, const double2 *__restrict__ pair,
                                                              const double2 *__restrict__ tw,
                                                              const uint32_t *__restrict__ task, int B,
                                                              FftGrid gd, double2 c8) {
    extern __shared__ double2 flds[];
    double2 *twl = flds + kFftM;
    for (int i = threadIdx.x; i < kFftTw; i += kFft4NT) twl[i] = tw[i];
    float2 v[2][16];
    {
        const int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units);
        const int c0 = fft_div(u, gd);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            fft_load_unit(p, c0, p.seg0 + (int64_t)(u - c0 * gd.nseg) * B, threadIdx.x + kFft4NT * h, v[h]);
    }
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    uint32_t tk_all[2] = {task[threadIdx.x], task[threadIdx.x + kFft4NT]};
    asm volatile("" : "+v"(tk_all[0]), "+v"(tk_all[1]));
    float pk_run = 0.0f;
    int pk_ch = -1;
    float *pk_lds = reinterpret_cast<float *>(twl + kFftTw);
    int pk_pending = -1;
    double2 wt[2][16];
#pragma unroll
    for (int h = 0; h < 2; ++h) powers16(twl[threadIdx.x + kFft4NT * h], wt[h]);
    int rnd = 0;
    for (int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units); u < gd.units;
         u = fft_unit32(++rnd, blockIdx.x, gridDim.x, gd.units)) {
    int jt = threadIdx.x;
    asm volatile("" : "+v"(jt));
    const int lane = jt & 63;
    const int wv = jt >> 6; // this kernel's wave (0..3); halves h = 0, 1 are 8-wave waves wv, wv + 4
    const int ch = fft_div(u, gd);
    const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;

    // ---- stage 1, both halves: thread b = jt + 256 h, 16-point DFT over z[512 a + b]
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        double2 a[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = make_double2((double)v[h][r].x, (double)v[h][r].y);
        dft16(a);
        apply16(a, wt[h]);
#pragma unroll
        for (int c = 0; c < 16; ++c) flds[512 * fft_slot(c) + jt + kFft4NT * h] = a[c];
    }
    __syncthreads();
    if (pk_pending >= 0) {
        if (threadIdx.x == 0) fft4_peak_commit(p, pk_pending, pk_lds);
        pk_pending = -1;
    }

    // four columns per wave: xa = column pairs of half 0 (x[0], x[1]) and half 1 (x[2], x[3])
    double2 x[4][8];
    double2 tws[8];
    double2 *blk[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        blk[2 * h] = flds + 512 * (2 * (wv + 4 * h));
        blk[2 * h + 1] = blk[2 * h] + 512;
    }
    const int l1 = lane & 7, d1s = lane >> 3;
    // ---- stage A: lane l holds b = l + 64 t; radix-8 over t -> d1; * W_512^(l d1)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int t = 0; t < 8; ++t) x[k][t] = blk[k][lane + 64 * t];
    powers8(twl[512 + lane], tws);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        dft8(x[k]);
        twiddle8(x[k], tws);
#pragma unroll
        for (int d1 = 0; d1 < 8; ++d1) blk[k][fx1(lane, d1)] = x[k][d1];
        wave_lds_sync();
#pragma unroll
        for (int l2 = 0; l2 < 8; ++l2) x[k][l2] = blk[k][fx1(l1 + 8 * l2, d1s)];
        __builtin_amdgcn_sched_barrier(0);
    }
    // ---- stage B: lane (l1, d1) has gathered l2; radix-8 -> e1; * W_64^(l1 e1)
    powers8(twl[512 + 8 * l1], tws);
    double2 tws_b[8];
    if constexpr (kOut == kFftOutSym) {
#pragma unroll
        for (int r = 1; r < 8; ++r) tws_b[r] = tws[r];
    }
    // ---- pair-table loads for both halves, ahead of stage C
    Fft4Pair<kOut> q[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) fft4_pair_load<kOut>(q[h], pair, jt + kFft4NT * h);
    __builtin_amdgcn_sched_barrier(0);
    // ---- stage C's tasks (per half): task A (cA, dA, eA), task B (cB, dB, eB)
    uint32_t tk[2] = {tk_all[0], tk_all[1]};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int k = 2 * h; k < 2 * h + 2; ++k) {
            dft8(x[k]);
            twiddle8(x[k], tws);
#pragma unroll
            for (int e1 = 0; e1 < 8; ++e1) blk[k][fx2(l1, d1s, e1)] = x[k][e1];
            __builtin_amdgcn_sched_barrier(0);
        }
        wave_lds_sync();
        // this half's stage-C reads, covered by the other half's stage B
        const int cA = tk[h] & 15, dA = (tk[h] >> 4) & 7, eA = (tk[h] >> 7) & 7;
        const int cB = (tk[h] >> 10) & 15, dB = (tk[h] >> 14) & 7, eB = (tk[h] >> 17) & 7;
        const double2 *ba = flds + 512 * cA, *bb = flds + 512 * cB;
#pragma unroll
        for (int l = 0; l < 8; ++l) x[2 * h][l] = ba[fx2(l, dA, eA)];
#pragma unroll
        for (int l = 0; l < 8; ++l) x[2 * h + 1][l] = bb[fx2(l, dB, eB)];
        __builtin_amdgcn_sched_barrier(0);
    }
    // ---- stage C + pair step + inverse stage A', per half
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        dft8(x[2 * h]);
        dft8(x[2 * h + 1]);
        fft4_pair<kOut>(x[2 * h], x[2 * h + 1], q[h], wv + 4 * h, lane, c8);
        const int cA = tk[h] & 15, dA = (tk[h] >> 4) & 7, eA = (tk[h] >> 7) & 7;
        const int cB = (tk[h] >> 10) & 15, dB = (tk[h] >> 14) & 7, eB = (tk[h] >> 17) & 7;
        double2 *ba = flds + 512 * cA, *bb = flds + 512 * cB;
        powers8(twl[512 + dA + 8 * eA], tws);
        dft8(x[2 * h]);
        twiddle8(x[2 * h], tws);
#pragma unroll
        for (int b0 = 0; b0 < 8; ++b0) ba[fx3(dA, eA, b0)] = x[2 * h][b0];
        __builtin_amdgcn_sched_barrier(0);
        powers8(twl[512 + dB + 8 * eB], tws);
        dft8(x[2 * h + 1]);
        twiddle8(x[2 * h + 1], tws);
#pragma unroll
        for (int b0 = 0; b0 < 8; ++b0) bb[fx3(dB, eB, b0)] = x[2 * h + 1][b0];
        __builtin_amdgcn_sched_barrier(0);
    }
    // ---- prefetch the next unit's samples (both halves)
    {
        const int un1 = fft_unit32(rnd + 1, blockIdx.x, gridDim.x, gd.units);
        const int un = un1 < gd.units ? un1 : u;
        const int cn = fft_div(un, gd);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            fft_load_unit(p, cn, p.seg0 + (int64_t)(un - cn * gd.nseg) * B, jt + kFft4NT * h, v[h]);
    }
    wave_lds_sync();
    // ---- stage B': lane (d1, beta0) gathers e1; radix-8 -> gamma0; * W_64^(gamma0 d1)
    {
        const int d1 = lane & 7, b0 = lane >> 3;
        const int rb0 = lane & 7, rg0 = lane >> 3;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e1 = 0; e1 < 8; ++e1) x[k][e1] = blk[k][fx3(d1, e1, b0)];
        if constexpr (kOut == kFftOutSym) {
#pragma unroll
            for (int r = 1; r < 8; ++r) tws[r] = tws_b[r];
        } else {
            powers8(twl[512 + 8 * d1], tws);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            dft8(x[k]);
            twiddle8(x[k], tws);
#pragma unroll
            for (int g0 = 0; g0 < 8; ++g0) blk[k][fx4(d1, b0, g0)] = x[k][g0];
            wave_lds_sync();
#pragma unroll
            for (int dd = 0; dd < 8; ++dd) x[k][dd] = blk[k][fx4(dd, rb0, rg0)];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // ---- stage C': lane rho = beta0 + 8 gamma0 has gathered d1; radix-8 -> gamma1
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        dft8(x[k]);
#pragma unroll
        for (int g1 = 0; g1 < 8; ++g1) blk[k][lane + 64 * g1] = x[k][g1];
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();

    // ---- final, per half: thread b gathers its 16 columns, * W_8192^(b c), 16-point DFT
    __builtin_amdgcn_s_waitcnt(kVmcnt0); // the prefetch has landed long ago
    float pk = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int jh = jt + kFft4NT * h;
        double2 a[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = flds[512 * fft_slot(c) + jh];
        powers16(twl[jh], wt[h]);
        apply16(a, wt[h]);
        dft16(a);
        pk = fmaxf(pk, fft4_store<kOut>(p, a, jh, ch, n0, B));
    }
    if (ch != pk_ch) {
        if (p.peak && pk_ch >= 0) {
            fft4_peak_stage(pk_lds, pk_run);
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
        if (pk_pending >= 0 && threadIdx.x == 0) fft4_peak_commit(p, pk_pending, pk_lds);
        __syncthreads();
        fft4_peak_stage(pk_lds, pk_run);
        __syncthreads();
        if (threadIdx.x == 0) fft4_peak_commit(p, pk_ch, pk_lds);
    }
}

} // namespace lcfir

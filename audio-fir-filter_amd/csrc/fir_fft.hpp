// fir_fft.hpp -- f64 overlap-save FFT evaluation of the FilterCore.h hot path.
//
// Same contract as fir_direct.hpp (y[n] = sum_k h[k] x[n - half + k], zero
// padding outside [0,N), outputs [start,end), RNE to f32), evaluated with
// f64 FFTs instead of T multiply-adds per sample.
//
// One workgroup = one segment of B = L - T + 1 consecutive outputs:
//   x_seg[i] = x[n0 - half + i], i in [0, L), L = 16384 real samples
//   c = IFFT_L( FFT_L(x_seg) * G ),  G = FFT_L(reversed taps, zero padded)
//   y[n0 + m - (T-1)] = c[m] for m in [T-1, L)          (overlap-save)
// The real length-L transform is done as one complex M = L/2 = 8192-point FFT
// of z[k] = x[2k] + i x[2k+1] with the even/odd split/merge fused into a
// single "pair" pass that also multiplies by G; the inverse uses the conj
// trick (IFFT(V) = conj(FFT(conj(V)))), so one forward Stockham kernel body
// (radix 16, 16, 16, 2) serves both directions.  All scale factors (the two
// 1/2 of the split/merge and the 1/M of the inverse) are folded into G, which
// the host computes once per filter in long double.
//
// Layout: the complex work array (8192 x 16 B = 128 KiB) lives in LDS with
// one pad slot per 16 entries (139 KiB), so one 512-thread workgroup fits a
// CU (2 waves per SIMD); each thread owns 16 complex values per pass.  The
// grid is persistent (one workgroup per CU looping over (channel, segment)
// units).  Samples are read and results written through range-checked raw
// buffer resources, so the zero padding at the channel edges and the output
// range clipping need no branches.  Twiddles of the inner passes come from a
// 1024-entry W_16384 table (L1-resident) raised to the needed powers in
// registers by a short odd/even product chain.
//
// Measured (profiles/): VALU ~25 %, LDS ~20 % busy; the
// binding cost is the barrier-serialised read -> compute -> write phases of
// the eight Stockham passes.  Persistence, prefetching the next unit's
// samples and hoisting the pair-pass loads were each measured neutral or
// negative; the next step is wave-local exchanges (fewer block barriers).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "fir_direct.hpp"

namespace lcfir {

constexpr int kFftL = 16384;        // real segment length
constexpr int kFftM = kFftL / 2;    // complex FFT length
constexpr int kFftNT = 512;         // threads per workgroup
constexpr int kFftTwN = 1024;       // entries of the W_L twiddle table
constexpr int kFftMinB = 2048;      // smallest useful segment (B = L - T + 1)

struct FftPlan {
    bool ready = false;
    int ntaps = 0;
    int B = 0;
    double2 *d_G = nullptr;  // M + 1 bins, scaled by 1 / (4M)
    double2 *d_tw = nullptr; // W_L^i, i in [0, kFftTwN)
    int cus = 256;           // compute units of the plan's device (persistent grid)
};

inline bool fft_supported(int ntaps) { return ntaps >= 1 && kFftL - ntaps + 1 >= kFftMinB; }
inline bool fft_preferred(int ntaps) { return ntaps >= 96 && fft_supported(ntaps); }

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {
    return make_double2(__builtin_fma(a.x, b.x, a.y * b.y), __builtin_fma(a.y, b.x, -(a.x * b.y)));
}
__device__ __forceinline__ double2 mul_mi(double2 a) { return make_double2(a.y, -a.x); } // * (-i)
__device__ __forceinline__ double2 mul_pi(double2 a) { return make_double2(-a.y, a.x); } // * (+i)

__device__ __forceinline__ int fpad(int i) { return i + (i >> 4); }

constexpr double kC1 = 0.92387953251128675613; // cos(pi/8)
constexpr double kS1 = 0.38268343236508977173; // sin(pi/8)
constexpr double kR2 = 0.70710678118654752440; // sqrt(1/2)

// forward radix-4 DFT in place (W4 = -i)
__device__ __forceinline__ void dft4(double2 &a0, double2 &a1, double2 &a2, double2 &a3) {
    const double2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_mi(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

// multiply by W16^m (forward, e^{-2 pi i m / 16}) for the m used by dft16
template <int m>
__device__ __forceinline__ double2 w16(double2 a) {
    if constexpr (m == 0) return a;
    else if constexpr (m == 1) return cmul(a, make_double2(kC1, -kS1));
    else if constexpr (m == 2) return make_double2(kR2 * (a.x + a.y), kR2 * (a.y - a.x));
    else if constexpr (m == 3) return cmul(a, make_double2(kS1, -kC1));
    else if constexpr (m == 4) return mul_mi(a);
    else if constexpr (m == 6) return make_double2(kR2 * (a.y - a.x), -kR2 * (a.x + a.y));
    else if constexpr (m == 9) return cmul(a, make_double2(-kC1, kS1));
    else static_assert(m == 0, "unused twiddle");
}

// forward 16-point DFT, natural order in and out (4 x 4 Cooley-Tukey)
__device__ __forceinline__ void dft16(double2 (&a)[16]) {
    // radix-4 over n1 for each n2: slot 4*n1 + n2 -> slot 4*k1 + n2
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(a[n2], a[4 + n2], a[8 + n2], a[12 + n2]);
    // twiddles W16^(n2*k1), slot 4*k1 + n2
    a[5] = w16<1>(a[5]);
    a[6] = w16<2>(a[6]);
    a[7] = w16<3>(a[7]);
    a[9] = w16<2>(a[9]);
    a[10] = w16<4>(a[10]);
    a[11] = w16<6>(a[11]);
    a[13] = w16<3>(a[13]);
    a[14] = w16<6>(a[14]);
    a[15] = w16<9>(a[15]);
    // radix-4 over n2 for each k1: slot 4*k1 + k2 holds X[k1 + 4*k2]
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) dft4(a[4 * k1], a[4 * k1 + 1], a[4 * k1 + 2], a[4 * k1 + 3]);
    double2 t[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) t[k1 + 4 * k2] = a[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = t[i];
}

// w[r] = w1^r for r = 1..15 by a product tree (depth <= 4)
__device__ __forceinline__ void twiddle_powers(double2 w1, double2 (&w)[16]) {
    w[1] = w1;
    w[2] = cmul(w1, w1);
    w[3] = cmul(w[2], w1);
    w[4] = cmul(w[2], w[2]);
    w[5] = cmul(w[4], w1);
    w[6] = cmul(w[4], w[2]);
    w[7] = cmul(w[4], w[3]);
    w[8] = cmul(w[4], w[4]);
#pragma unroll
    for (int r = 9; r < 16; ++r) w[r] = cmul(w[8], w[r - 8]);
}

// Second half of a Stockham radix-16 pass (N = 8192, 512 butterflies, one per
// thread): twiddle, DFT16, store to LDS in expanded order.
template <int NS>
__device__ __forceinline__ void r16_finish(double2 (&a)[16], double2 *lds, int j, double2 w1) {
    if constexpr (NS > 1) {
        // w1 = W_{NS*16}^(j % NS); element r is multiplied by w1^r.  Powers by
        // an odd/even chain (w^(2i+1) = w^(2i-1) w^2): 4 live values instead of
        // a 15-entry table, <= 8 products deep (error ~1e-15).
        const double2 w2 = cmul(w1, w1);
        double2 wo = w1, we = w2;
        a[1] = cmul(a[1], wo);
        a[2] = cmul(a[2], we);
#pragma unroll
        for (int r = 3; r < 15; r += 2) {
            wo = cmul(wo, w2);
            we = cmul(we, w2);
            a[r] = cmul(a[r], wo);
            a[r + 1] = cmul(a[r + 1], we);
        }
        a[15] = cmul(a[15], cmul(wo, w2));
    }
    dft16(a);
    const int idx = (j / NS) * NS * 16 + (j % NS);
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[fpad(idx + r * NS)] = a[r];
}

template <int NS>
__device__ __forceinline__ void r16_pass(double2 *lds, int j, double2 w1) {
    double2 a[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = lds[fpad(j + r * (kFftM / 16))];
    __syncthreads(); // every read of this pass before any write (in place)
    r16_finish<NS>(a, lds, j, w1);
    __syncthreads();
}

// constant W_16^q and W_32^q (forward)
__device__ __forceinline__ double2 w16q(int q) {
    constexpr double c[8] = {1.0, kC1, kR2, kS1, 0.0, -kS1, -kR2, -kC1};
    constexpr double s[8] = {0.0, kS1, kR2, kC1, 1.0, kC1, kR2, kS1};
    return make_double2(c[q], -s[q]);
}

__device__ __forceinline__ double2 w32q(int q) {
    constexpr double c[8] = {1.0, 0.98078528040323044913, kC1, 0.83146961230254523708,
                             kR2, 0.55557023301960222474, kS1, 0.19509032201612826785};
    constexpr double s[8] = {0.0, 0.19509032201612826785, kS1, 0.55557023301960222474,
                             kR2, 0.83146961230254523708, kC1, 0.98078528040323044913};
    return make_double2(c[q], -s[q]);
}

// Final radix-2 pass (NS = 4096) of the 8192-point transform: thread j owns
// butterflies b = j + 512 q, q < 8; lo[q] = X[b], hi[q] = X[b + 4096].
__device__ __forceinline__ void r2_pass(const double2 *lds, int j, double2 wj /* W_8192^j */,
                                        double2 (&lo)[8], double2 (&hi)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int b = j + 512 * q;
        const double2 v0 = lds[fpad(b)];
        double2 v1 = lds[fpad(b + kFftM / 2)];
        // W_8192^b = W_8192^j * W_16^q
        const double2 w = (q == 0) ? wj : cmul(wj, w16q(q));
        v1 = cmul(v1, w);
        lo[q] = cadd(v0, v1);
        hi[q] = csub(v0, v1);
    }
}

// Split/merge of the real transform fused with the filter multiply.
// In: Zk = Z[k], Zmk = Z[M-k], W = W_L^k.  Out: V[k], V[M-k] (scaled by 4M,
// folded into G).
__device__ __forceinline__ void pair_step(double2 Zk, double2 Zmk, double2 W, double2 Gk,
                                          double2 Gmk, double2 &Vk, double2 &Vmk) {
    const double2 Zm = cconj(Zmk);
    const double2 E = cadd(Zk, Zm);
    const double2 O = mul_mi(csub(Zk, Zm));
    const double2 WO = cmul(W, O);
    const double2 Xk = cadd(E, WO);
    const double2 Xmk = cconj(csub(E, WO));
    const double2 Yk = cmul(Xk, Gk);
    const double2 Ymk = cmul(Xmk, Gmk);
    const double2 Ep = cadd(Yk, cconj(Ymk));
    const double2 Op = cmulc(csub(Yk, cconj(Ymk)), W);
    Vk = cadd(Ep, mul_pi(Op));
    Vmk = cadd(cconj(Ep), mul_pi(cconj(Op)));
}

// Samples of one unit: v[r] = (x_seg[2m], x_seg[2m+1]), m = j + 512 r, x_seg[i] =
// x[n0 - half + i].  Raw buffer loads through a range-checked resource over the
// loaded window [x_lo, x_hi): offsets outside it -- including "negative" ones,
// which wrap to huge unsigned offsets -- read 0.  That is the zero padding of
// FilterCore.h's shortened edge sums, with no branches.
__device__ __forceinline__ void fft_load_unit(const DirectParams &p, int ch, int64_t n0, int j,
                                              float2 (&v)[16]) {
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(x), (short)0, (int)((p.x_hi - p.x_lo) * 4), 0x00020000);
    const int off0 = (int)((n0 - p.half - p.x_lo) * 4) + 8 * j; // may be negative
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int off = off0 + 8 * 512 * r;
        // aux bit 31 = volatile: keeps the two dword loads from being merged
        // into one dwordx2, whose range check is all-or-nothing (a pair
        // straddling the window start would lose its in-range sample)
        v[r].x = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, (int)0x80000000));
        v[r].y = __int_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, (int)0x80000000));
    }
}

// Persistent: one workgroup per CU walks the units u = blockIdx.x + i * gridDim.x
// of the nch x nseg (channel, segment) grid, so no CU idles between workgroup
// dispatches.
__global__ __launch_bounds__(kFftNT) void fir_fft_f64_kernel(DirectParams p, const double2 *__restrict__ G,
                                                            const double2 *__restrict__ tw, int B,
                                                            int64_t nseg, int64_t units) {
    extern __shared__ double2 flds[];
    for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
    // Laundered thread index: everything derived from it (twiddles, LDS
    // addresses) is recomputed per unit instead of being hoisted out of the
    // loop, which would keep hundreds of values live and spill.
    int j = threadIdx.x;
    asm volatile("" : "+v"(j));
    const int ch = (int)(u / nseg);
    const int64_t n0 = p.start + (u % nseg) * B;

    // ---- forward pass 1 (NS = 1): z[m] = (x_seg[2m], x_seg[2m+1]), m = j + 512 r
    {
        float2 v[16];
        fft_load_unit(p, ch, n0, j, v);
        double2 a[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = make_double2((double)v[r].x, (double)v[r].y);
        r16_finish<1>(a, flds, j, make_double2(1.0, 0.0));
        __syncthreads();
    }
    r16_pass<16>(flds, j, tw[2 * ((j % 16) * (kFftM / 256))]);
    r16_pass<256>(flds, j, tw[2 * ((j % 256) * (kFftM / 4096))]);

    // ---- forward radix-2 pass; upper half goes to LDS for the partner thread
    double2 lo[8], hi[8];
    r2_pass(flds, j, tw[2 * j], lo, hi);
#pragma unroll
    for (int q = 0; q < 8; ++q) flds[fpad(j + 512 * q + kFftM / 2)] = hi[q];
    __syncthreads();

    // ---- pair pass: V[k], V[M-k] for k = j + 512 q (< M/2), plus k = M/2 (thread 0)
    {
        const double2 wj = tw[j]; // W_L^j
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int k = j + 512 * q;
            const double2 Zk = lo[q];
            const double2 Zmk = (k == 0) ? Zk : flds[fpad(kFftM - k)];
            // W_L^k = W_L^j * W_32^q
            const double2 W = (q == 0) ? wj : cmul(wj, w32q(q));
            double2 Vk, Vmk;
            pair_step(Zk, Zmk, W, G[k], G[kFftM - k], Vk, Vmk);
            flds[fpad(k)] = Vk;
            if (k != 0) flds[fpad(kFftM - k)] = Vmk;
        }
        if (j == 0) {
            const int k = kFftM / 2;
            const double2 Zk = flds[fpad(k)];
            double2 Vk, Vmk;
            pair_step(Zk, Zk, make_double2(0.0, -1.0), G[k], G[k], Vk, Vmk);
            flds[fpad(k)] = Vk;
        }
    }
    __syncthreads();

    // ---- inverse: conj(FFT(conj(V)))
    {
        double2 a[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = cconj(flds[fpad(j + 512 * r)]);
        __syncthreads();
        r16_finish<1>(a, flds, j, make_double2(1.0, 0.0));
        __syncthreads();
    }
    r16_pass<16>(flds, j, tw[2 * ((j % 16) * (kFftM / 256))]);
    r16_pass<256>(flds, j, tw[2 * ((j % 256) * (kFftM / 4096))]);
    r2_pass(flds, j, tw[2 * j], lo, hi);

    // ---- outputs: c[2m] = Re v'[m], c[2m+1] = -Im v'[m], valid for 2m+e >= T-1
    // Range-checked buffer over y[start, end): invalid lanes store to an
    // out-of-range offset, which the hardware drops (no branches).  c index
    // < T-1 belongs to the previous segment; beyond `end` is outside the range.
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
        yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
    const int cmin = p.ntaps - 1;
    const int64_t off = n0 - cmin - p.start; // offset (samples) of c[0] from start
    const int64_t oend = p.end - p.start;
    float pk = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int c = 2 * (j + 512 * q + h * (kFftM / 2));
            const double2 v = h ? hi[q] : lo[q];
            const float f0 = (float)v.x, f1 = (float)(-v.y);
            const int64_t o = off + c;
            const bool ok0 = c >= cmin && o < oend, ok1 = c + 1 >= cmin && o + 1 < oend;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys,
                                                  ok0 ? (int)(o * 4) : (int)0x80000000, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                  ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, 0);
            pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
        }
    }
    if (p.peak) {
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) pk = fmaxf(pk, __shfl_xor(pk, s, 64));
        if ((j & 63) == 0) atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(pk));
    }
    __syncthreads(); // the next unit's first LDS writes follow this unit's last reads
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace detail {
// in-place iterative radix-2 complex FFT in long double (forward, e^{-i...})
inline void fft_ld(std::vector<long double> &re, std::vector<long double> &im) {
    const size_t n = re.size();
    for (size_t i = 1, jj = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; jj & bit; bit >>= 1) jj ^= bit;
        jj ^= bit;
        if (i < jj) {
            std::swap(re[i], re[jj]);
            std::swap(im[i], im[jj]);
        }
    }
    const long double two_pi = 6.283185307179586476925286766559L;
    for (size_t len = 2; len <= n; len <<= 1) {
        const size_t h = len >> 1;
        for (size_t k = 0; k < h; ++k) {
            const long double a = -two_pi * (long double)k / (long double)len;
            const long double wr = cosl(a), wi = sinl(a);
            for (size_t s = 0; s < n; s += len) {
                const size_t u = s + k, v = s + k + h;
                const long double tr = re[v] * wr - im[v] * wi;
                const long double ti = re[v] * wi + im[v] * wr;
                re[v] = re[u] - tr;
                im[v] = im[u] - ti;
                re[u] += tr;
                im[u] += ti;
            }
        }
    }
}
} // namespace detail

inline bool fft_plan_build(FftPlan &plan, const double *d_taps, int ntaps, hipStream_t s,
                           std::string &err) {
    if (!fft_supported(ntaps)) {
        err = "tap count too large for the L=16384 overlap-save segment";
        return false;
    }
    std::vector<double> taps((size_t)ntaps);
    if (hipMemcpy(taps.data(), d_taps, sizeof(double) * (size_t)ntaps, hipMemcpyDeviceToHost) !=
        hipSuccess) {
        err = "tap download failed";
        return false;
    }
    // G = FFT_L(g), g[j] = h[T-1-j], zero padded; scaled by 1/(4M)
    std::vector<long double> re((size_t)kFftL, 0.0L), im((size_t)kFftL, 0.0L);
    for (int i = 0; i < ntaps; ++i) re[(size_t)i] = (long double)taps[(size_t)(ntaps - 1 - i)];
    detail::fft_ld(re, im);
    std::vector<double2> G((size_t)kFftM + 1);
    const long double scale = 1.0L / (4.0L * (long double)kFftM);
    for (int k = 0; k <= kFftM; ++k)
        G[(size_t)k] = make_double2((double)(re[(size_t)k] * scale), (double)(im[(size_t)k] * scale));
    std::vector<double2> tw((size_t)kFftTwN);
    const long double two_pi = 6.283185307179586476925286766559L;
    for (int i = 0; i < kFftTwN; ++i) {
        const long double a = -two_pi * (long double)i / (long double)kFftL;
        tw[(size_t)i] = make_double2((double)cosl(a), (double)sinl(a));
    }
    if (hipMalloc(reinterpret_cast<void **>(&plan.d_G), sizeof(double2) * G.size()) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&plan.d_tw), sizeof(double2) * tw.size()) != hipSuccess) {
        err = "hipMalloc for the FFT plan failed";
        return false;
    }
    if (hipMemcpy(plan.d_G, G.data(), sizeof(double2) * G.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(plan.d_tw, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice) !=
            hipSuccess) {
        err = "FFT plan upload failed";
        return false;
    }
    (void)s;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        cus > 0)
        plan.cus = cus;
    plan.ntaps = ntaps;
    plan.B = kFftL - ntaps + 1;
    plan.ready = true;
    return true;
}

constexpr size_t fft_lds_bytes() { return sizeof(double2) * (size_t)(kFftM + kFftM / 16); }

// workgroups per CU the persistent grid assumes (139 KiB of LDS each: one);
// LCFIR_FFT_BLOCKS_PER_CU overrides for experiments
inline int fft_blocks_per_cu() {
    static const int v = [] {
        const char *e = std::getenv("LCFIR_FFT_BLOCKS_PER_CU");
        const int b = e ? std::atoi(e) : 1;
        return b > 0 ? b : 1;
    }();
    return v;
}

inline bool fft_launch(const FftPlan &plan, const DirectParams &p, int nch, hipStream_t s,
                       std::string &err) {
    const int64_t count = p.end - p.start;
    if (count <= 0 || nch <= 0) return true;
    const int64_t nseg = (count + plan.B - 1) / plan.B;
    if (nseg > 0x7fffffff || nch > 65535) {
        err = "range too large for one launch";
        return false;
    }
    static bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(&fir_fft_f64_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)fft_lds_bytes()) == hipSuccess;
    }();
    (void)attr;
    const int64_t units = nseg * nch;
    const int64_t grid = std::min<int64_t>(units, (int64_t)plan.cus * fft_blocks_per_cu());
    hipLaunchKernelGGL(fir_fft_f64_kernel, dim3((unsigned)grid), dim3(kFftNT), fft_lds_bytes(), s,
                       p, plan.d_G, plan.d_tw, plan.B, nseg, units);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        err = hipGetErrorString(e);
        return false;
    }
    return true;
}

inline void fft_plan_free(FftPlan &plan) {
    if (plan.d_G) (void)hipFree(plan.d_G);
    if (plan.d_tw) (void)hipFree(plan.d_tw);
    plan = FftPlan{};
}

} // namespace lcfir

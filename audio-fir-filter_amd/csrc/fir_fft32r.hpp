// fir_fft32r.hpp -- the L = 32 768 zero-phase overlap-save unit held in
// registers (its history: CHANGELOG.md s4.2).
//
// fir_fft32.hpp runs an L = 32 768 segment as two 8192-point halves through
// fir_fft.hpp's column phase, parking the idle half in a global slab: 12 LDS
// round trips of 128 KiB per segment, the same LDS bytes per transform point
// as L = 16 384.  Here the 16 384-point complex transform stays in the
// register file instead -- 32 complex f64 per thread, 256 KiB per workgroup,
// half of the CU's VGPRs -- and the LDS only carries the exchanges, each in
// two rounds of 128 KiB:
//
//   z[m] = x_seg[2m] + i x_seg[2m+1], m = 512 n + b (thread b, register n),
//   b = 16 beta + gamma;   bins k = k1 + 32 kappa + 1024 lambda.
//   stage 1 (thread b): DFT32 over n -> k1, * W_16384^(b k1)
//   T1 (workgroup, 2 rounds): lane (k1, gamma) of column k1 gathers beta
//   stage 2: DFT32 over beta -> kappa, * W_512^(gamma kappa)
//   T2 (wave-local, 2 rounds): lane s of a 32-lane group gathers gamma for
//       task R1 (column, kappa < 16) and task R2 (its mirror, kappa >= 16)
//   stage 3: DFT16 over gamma -> lambda;  pair step R1[i] <-> R2[15 - i]
//   (bins k and N - k), the zero-phase pair table; then stage 3, T2, stage 2,
//   T1 and stage 1 again in reverse (the inverse as conj(FFT(conj(V)))).
// Per segment: 4 exchanges (8 LDS rounds) of 256 KiB against fir_fft32.hpp's
// 12 round trips of 128 KiB, 6 workgroup barriers, 3 radix stages per
// direction instead of 4.
//
// Every register index is the same in every lane (no lane-dependent register
// selection, which the compiler would lower through scratch):
//   * round 1 of T1 carries the columns k1 < 16 of threads b < 256 and the
//     columns k1 >= 16 of threads b >= 256.  Waves 4..7 negate their odd
//     stage-1 inputs, which rotates their DFT32 outputs by 16 (register r
//     holds k1 = r + 16 mod 32), so round 1 is registers 0..15 everywhere.
//   * a column lane with k1 >= 16 (h = 1) receives beta rotated by 16; its
//     DFT32 output picks up (-1)^kappa, folded into the twiddle base
//     (-W_512^gamma instead of W_512^gamma).  The inverse stage 2 uses the same
//     base, which rotates its outputs back into the round order.
//   * the final DFT32 of waves 4..7 sees k1 rotated by 16: (-1)^n on its
//     outputs, folded into the f32 stores' sign bits.
// Wave 0's lane 31 holds the self-paired bins 0 and N/2 (tasks (0, 0) and
// (0, 16)); it permutes its registers through a 512-B LDS scratch before and
// after the pair step (per-lane select chains in place spilled VGPRs).  scripts/fft32r_model.py is the numpy model of this
// flow (every register index, LDS slot and table slot; bank conflicts).
//
// Included by fir_fft.hpp after fir_fft32.hpp, inside namespace lcfir.

constexpr int kR32TwB = 0;      // W_16384^b, b < 512
constexpr int kR32TwB16 = 512;  // W_1024^b = W_16384^(16 b), b < 512
constexpr int kR32TwG = 1024;   // W_512^g, g < 16
constexpr int kR32Tw = 1024 + 16;
constexpr size_t kR32PairTable = (size_t)24 * kFftNT; // double2: (p1, q2) [16][512], (p2 even, p2 odd) [8][512]
constexpr int kR32SpecialLane = 31;                   // of wave 0
// Instrumentation hook: the kernel calls Probe::stamp(i, rnd) at each phase
// boundary i of its unit rnd.  The product's probe does nothing;
// tools/fft32r_trace.hip passes one that records s_memtime.
struct R32NoProbe {
    __device__ static void stamp(int, int) {}
};

// The pair path's output stores: one vector-memory instruction per register
// pair, issued after the next unit's split LDS-DMA (r32_dma_part).  The next
// unit's top waits vmcnt(kR32PairStores): the DMA has landed once at most the
// stores issued after it are still in flight.  That holds only if no other
// vector-memory instruction (a scratch spill or reload included) is issued
// between the DMA and the next unit's top; the build checks every
// fir_fft32r_kernel for zero scratch (Makefile `check-scratch`).
constexpr int kR32PairStores = 32;
// s_waitcnt immediate for vmcnt(n), expcnt and lgkmcnt left at their maxima
constexpr int r32_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }
static_assert(kR32PairStores < 64 && r32_vmcnt(kR32PairStores) == 0x8F70 && r32_vmcnt(0) == kVmcnt0,
              "vmcnt(n) encoding: low 4 bits in [3:0], high 2 bits in [15:14]");

// LDS work array: one region per wave (T1 / T1 backwards address regions by
// wave; T2 stays inside its wave's region), 32-lane groups and halves inside
// T2's rows are padded to 17 slots: conflict-free without an XOR swizzle's
// address math (-5 %)
constexpr int kR32Row = 17;
constexpr int kR32Hs = 16 * kR32Row;  // double2 per 32-lane half (16 rows)
constexpr int kR32Gs = 2 * kR32Hs;    // per 32-lane group
constexpr int kR32Rg = 2 * kR32Gs;    // per wave region
constexpr int kR32Work = 8 * kR32Rg;
// T2 slot of (half base, kappa mod 16, gamma): conflict-free for the writers
// (8 consecutive gamma) and the readers (16 distinct kappa per read group)
__device__ __forceinline__ int r32_t2(int base, int kl, int gam) { return base + kR32Row * kl + gam; }
// a T2 reader's slot for register i = gamma; rb = its half base + row offset
__device__ __forceinline__ int r32_t2r(int rb, int i) { return rb + i; }

// column k1 of lane (wave w, 32-lane group g, half h); mirror columns k1 and
// 32 - k1 share a group (wave 0 group 0: the self-paired columns 0 and 16)
__host__ __device__ constexpr int r32_column(int w, int g, int h) {
    return w == 0 ? (g ? (h ? 24 : 8) : (h ? 16 : 0)) : (g ? (h ? 24 - w : w + 8) : (h ? 32 - w : w));
}
// 4 wave + 2 g + h of column k1 (the inverse of r32_column)
__host__ __device__ constexpr int r32_column_home(int k1) {
    return k1 == 0 ? 0 : k1 == 16 ? 1 : k1 == 8 ? 2 : k1 == 24 ? 3
         : k1 < 8 ? 4 * k1 : k1 > 24 ? 4 * (32 - k1) + 1 : k1 < 16 ? 4 * (k1 - 8) + 2 : 4 * (24 - k1) + 3;
}

// Task word of thread t (host): T2's read tasks (h, kappa mod 16) for R1 (bits
// 0..4) and R2 (bits 5..9), scripts/fft32r_model.py's t2_tasks
inline uint32_t r32_task_word(int t) {
    const int w = t >> 6, g = (t >> 5) & 1, s = t & 31;
    int h1, k1, h2, k2;
    if (w == 0 && g == 0) {
        // column 16's tasks on read group {0-3, 12-15, 20-27}, column 0's and
        // the special lane on {4-11, 16-19, 28-31}: conflict-free T2 reads
        static const int ga[16] = {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27};
        static const int gb[15] = {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30};
        int ia = -1, ib = -1;
        for (int i = 0; i < 16; ++i)
            if (ga[i] == s) ia = i;
        for (int i = 0; i < 15; ++i)
            if (gb[i] == s) ib = i;
        if (ia >= 0) {
            h1 = 1, k1 = ia, h2 = 1, k2 = 31 - ia;
        } else if (ib >= 0) {
            h1 = 0, k1 = 1 + ib, h2 = 0, k2 = 31 - ib;
        } else {
            h1 = 0, k1 = 0, h2 = 0, k2 = 16; // the special lane
        }
    } else if (s < 16) {
        h1 = 0, k1 = s, h2 = 1, k2 = 31 - s;
    } else {
        h1 = 1, k1 = 31 - s, h2 = 0, k2 = s;
    }
    return (uint32_t)(h1 | (k1 & 15) << 1 | h2 << 5 | (k2 & 15) << 6);
}
// bins of thread t's R1 / R2 registers lambda = 0..15 (host; pair tables)
inline void r32_task_bins(int t, int (&bx)[16], int (&by)[16]) {
    const int w = t >> 6, g = (t >> 5) & 1;
    const uint32_t tk = r32_task_word(t);
    const int cA = r32_column(w, g, tk & 1), kA = (tk >> 1) & 15;
    const int cB = r32_column(w, g, (tk >> 5) & 1), kB = 16 + ((tk >> 6) & 15);
    for (int l = 0; l < 16; ++l) {
        bx[l] = cA + 32 * kA + 1024 * l;
        by[l] = cB + 32 * kB + 1024 * l;
    }
}

// forward 16-point DFT with the W16 rotations in FMA form (fir_fft.hpp's
// rot16_* / dft4_r2c: tan(pi/8) rotations, cos(pi/8) folded into the row's
// radix-4): 8 f64 operations fewer than dft16
__device__ __forceinline__ void dft16f(double2 (&a)[16]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(a[n2], a[4 + n2], a[8 + n2], a[12 + n2]);
    a[10] = w16<4>(a[10]);
    dft4(a[0], a[1], a[2], a[3]);
    {
        double2 o1, o3;
        dft4_r2c(a[4], rot16_1(a[5]), rot8_1(a[6]), a[6], rot16_3(a[7]), o1, o3);
        a[5] = o1;
        a[7] = o3;
    }
    {
        double2 o1, o3;
        dft4_r13(a[8], rot8_1(a[9]), a[10], rot8_3(a[11]), o1, o3);
        a[9] = o1;
        a[11] = o3;
    }
    {
        double2 o1, o3;
        dft4_r2c(a[12], rot16_3(a[13]), rot8_3(a[14]), a[14], rot16_9(a[15]), o1, o3);
        a[13] = o1;
        a[15] = o3;
    }
    double2 t[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) t[k1 + 4 * k2] = a[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = t[i];
}

// W32^k = cos t - i sin t (t = pi k / 16) as f (1 - i r) with |r| <= 1: f = cos t,
// r = tan t where |cos| >= |sin|, else (-i) f (1 + i r) with f = sin t, r = cot t
constexpr double kW32Fac[16] = {1.0, 0.98078528040323044913, 0.92387953251128675613, 0.83146961230254523708,
                                0.70710678118654752440, 0.83146961230254523708, 0.92387953251128675613,
                                0.98078528040323044913, 1.0, 0.98078528040323044913, 0.92387953251128675613,
                                0.83146961230254523708, 0.70710678118654752440, 0.83146961230254523708,
                                0.92387953251128675613, 0.98078528040323044913};
constexpr double kW32Rat[16] = {0.0, 0.19891236737965800691, 0.41421356237309504880, 0.66817863791929891999,
                                1.0, 0.66817863791929891999, 0.41421356237309504880, 0.19891236737965800691,
                                0.0, -0.19891236737965800691, -0.41421356237309504880, -0.66817863791929891999,
                                -1.0, -0.66817863791929891999, -0.41421356237309504880, -0.19891236737965800691};

// forward 32-point DFT, natural order in and out: radix 2 over two DFT16s, each
// butterfly's W32^k rotation in FMA form (the factor f folded into the
// butterfly: 6 f64 operations per k instead of 8)
// (hook: called between the two DFT16s)
template <class Hook>
__device__ __forceinline__ void dft32_hook(double2 (&a)[32], Hook &&hook) {
    double2 e[16], o[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        e[r] = a[2 * r];
        o[r] = a[2 * r + 1];
    }
    dft16f(e);
    hook();
    dft16f(o);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k == 0 || k == 8) {
            const double2 t = k == 0 ? o[k] : mul_mi(o[k]);
            a[k] = cadd(e[k], t);
            a[k + 16] = csub(e[k], t);
            continue;
        }
        const double f = kW32Fac[k], r = kW32Rat[k];
        double2 q; // o W32^k / f
        if (k < 5 || k > 11) // cos-major: o (1 - i r) (k >= 12: cos < 0, the sign in fs)
            q = make_double2(__builtin_fma(r, o[k].y, o[k].x), __builtin_fma(-r, o[k].x, o[k].y));
        else // sin-major: (-i) o (1 + i r)
            q = make_double2(__builtin_fma(r, o[k].x, o[k].y), __builtin_fma(r, o[k].y, -o[k].x));
        const double fs = (k >= 12) ? -f : f; // cos t < 0 on the cos-major side past pi / 2
        a[k] = make_double2(__builtin_fma(fs, q.x, e[k].x), __builtin_fma(fs, q.y, e[k].y));
        a[k + 16] = make_double2(__builtin_fma(-fs, q.x, e[k].x), __builtin_fma(-fs, q.y, e[k].y));
    }
}
__device__ __forceinline__ void dft32(double2 (&a)[32]) {
    dft32_hook(a, [] {});
}

// a[off + r] *= s0 w^r, r < R (a multiple of 4), for a unit w, w4 = w^4:
// anchors A = s0 w^(4m) by complex multiplies, and from each anchor two
// Chebyshev steps s_(r+1) = 2 Re(w) s_r - s_(r-1) (two FMAs a power).  The
// plain recurrence over 31 powers amplifies rounding to ~6e-14 for small
// angles -- 14 f32 ulps at config 3's smallest outputs; two steps from an
// anchor stay at the chains' ~2e-15.  Each power is applied as it is made.
template <int R>
__device__ __forceinline__ void r32_chain_anchored(double2 (&a)[32], int off, double2 s0, double2 w, double2 w4) {
    const double c2 = w.x + w.x;
    double2 A = s0;
#pragma unroll
    for (int m = 0; m < R / 4; ++m) {
        const double2 p1 = cmul(A, w);
        const double2 p2 = make_double2(__builtin_fma(c2, p1.x, -A.x), __builtin_fma(c2, p1.y, -A.y));
        const double2 p3 = make_double2(__builtin_fma(c2, p2.x, -p1.x), __builtin_fma(c2, p2.y, -p1.y));
        a[off + 4 * m] = cmul(a[off + 4 * m], A);
        a[off + 4 * m + 1] = cmul(a[off + 4 * m + 1], p1);
        a[off + 4 * m + 2] = cmul(a[off + 4 * m + 2], p2);
        a[off + 4 * m + 3] = cmul(a[off + 4 * m + 3], p3);
        if (m + 1 < R / 4) A = cmul(A, w4);
    }
}
// a[r] *= w^r, r < 32
__device__ __forceinline__ void r32_chain32acc(double2 (&a)[32], double2 w) {
    const double2 w2 = cmul(w, w);
    const double2 w4 = cmul(w2, w2);
    const double c2 = w.x + w.x;
    // anchor 0 is 1: its powers w, 2 Re(w) w - 1, ...
    const double2 p2 = make_double2(__builtin_fma(c2, w.x, -1.0), c2 * w.y);
    const double2 p3 = make_double2(__builtin_fma(c2, p2.x, -w.x), __builtin_fma(c2, p2.y, -w.y));
    a[1] = cmul(a[1], w);
    a[2] = cmul(a[2], p2);
    a[3] = cmul(a[3], p3);
    r32_chain_anchored<28>(a, 4, w4, w, w4);
}
// stage 1 / final: register r holds k1 = r + 16 hi (mod 32): registers 0..15
// take s0 w^r, 16..31 s1 w^(r-16), {s0, s1} = {1, w16} (w16 = W_1024^b, a table value)
__device__ __forceinline__ void r32_chain_k1acc(double2 (&a)[32], double2 w, double2 w16, bool hi) {
    const double2 w2 = cmul(w, w);
    const double2 w4 = cmul(w2, w2);
    const double2 one = make_double2(1.0, 0.0);
    r32_chain_anchored<16>(a, 0, csel(hi, w16, one), w, w4);
    r32_chain_anchored<16>(a, 16, csel(hi, one, w16), w, w4);
}

// Samples of unit (ch, n0) into wave w's region flds[1024 w, + 1024) as the
// float2 z[512 n + 64 w + i] at float2 index 2048 w + 64 n + i (the caller
// has retired the wave's reads of its region).  Interior units by LDS-DMA
// (16 b128 transfers per lane, no VGPRs); edge units through fft_load_unit's
// range-checked loads.
// interior unit of channel ch at n0: its window lies inside [x_lo, x_hi)
__device__ __forceinline__ bool r32_interior(const DirectParams &p, int64_t n0) {
    const int64_t w0 = n0 - p.half - p.x_lo;
    return w0 >= 0 && w0 + kFft32L <= p.x_hi - p.x_lo;
}
// One LDS-DMA transfer (16 B per lane to LDS byte lds + 16 lane) issued by
// inline asm: the compiler then does not know it writes LDS, so it adds no
// vmcnt(0) before the next unit's LDS reads; the explicit vmcnt(kR32PairStores)
// at the next unit's top orders them instead (every later compiler wait only
// over-counts).
__device__ __forceinline__ void r32_dma_asm(const float *base, uint32_t nbytes, uint32_t lds, int vofs, int sofs) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const u4 rs = {(unsigned)a, (unsigned)(a >> 32) & 0xFFFFu, nbytes, 0x00020000u};
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm" // m0 is reserved; the compiler sets it before each of its own uses
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds), "v"(vofs), "s"(rs),
                 "s"(sofs)
                 : "memory", "m0");
#pragma clang diagnostic pop
}
// transfers [s0, s1) of an interior unit's LDS-DMA (r32_stage_samples)
template <int s0, int s1>
__device__ __forceinline__ void r32_dma_part(const DirectParams &p, int ch, int64_t n0, int j, double2 *flds) {
    const int w = j >> 6, lane = j & 63;
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const int64_t w0 = n0 - p.half - p.x_lo;
    const int vofs = 4096 * (lane >> 5) + 512 * w + 16 * (lane & 31);
    const int sofs = (int)(w0 * 4);
    // one address-space cast of the array base, the region offset in bytes
    // (casting each element pointer miscompiles in some instantiations)
    const uint32_t lds0 = (uint32_t)(size_t)(fft_lds_void *)flds;
#pragma unroll
    for (int s = s0; s < s1; ++s)
        r32_dma_asm(x, (uint32_t)((p.x_hi - p.x_lo) * 4),
                    __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(16 * (kR32Rg * w + 64 * s))), vofs,
                    sofs + 8192 * s);
}
__device__ __forceinline__ void r32_stage_samples(const DirectParams &p, int ch, int64_t n0, int j, double2 *flds) {
    const int w = j >> 6, lane = j & 63;
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const int64_t w0 = n0 - p.half - p.x_lo;
    if (w0 >= 0 && w0 + kFft32L <= p.x_hi - p.x_lo) {
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(x), (short)0, (int)((p.x_hi - p.x_lo) * 4), 0x00020000);
        // transfer s, lane l: z[512 n + 64 w + 2k], z[.. + 1], n = 2s + (l >> 5),
        // k = l & 31 (the 16 bytes at 4 w0 + 8192 s + 4096 (l >> 5) + 512 w + 16 k)
        // into LDS byte 16384 w + 1024 s + 16 l (float2 2048 w + 64 n + 2k)
        const int vofs = 4096 * (lane >> 5) + 512 * w + 16 * (lane & 31);
        const int sofs = (int)(w0 * 4);
#pragma unroll
        for (int s = 0; s < 16; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (fft_lds_void *)(flds + kR32Rg * w + 64 * s), 16, vofs,
                                                     sofs + 8192 * s, 0, 0);
    } else {
        float2 v[32];
        fft_load_unit<32>(p, ch, n0, j, v);
        float2 *fz = reinterpret_cast<float2 *>(flds) + 2 * kR32Rg * w + lane;
#pragma unroll
        for (int n = 0; n < 32; ++n) fz[64 * n] = v[n];
    }
}

// a unit whose outputs take the pair-store path (kR32PairStores per lane)
__device__ __forceinline__ bool r32_pair_path(const DirectParams &p, int64_t n0, int B) {
    return (p.half & 1) == 0 && n0 >= p.start && (p.end - n0 >= B || ((p.end - n0) & 1) == 0);
}

// Outputs of one unit: c[2m] = Re out[n], c[2m+1] = -Im out[n], m = j + 512 n,
// valid for c in [half, L - half); sg = the sign bit waves 4..7 put on odd n
// (their rotated final DFT32).  Range-checked buffer stores, nt: 8-byte pairs
// through a per-unit resource when half is even (r32_pair_path), else one
// dword per output with explicit range checks (an odd half or a unit that
// straddles the range's start).
__device__ __forceinline__ float r32_store_unit(const DirectParams &p, int ch, int64_t n0, int B, int j,
                                                const double2 (&o)[32], int sg) {
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const __amdgpu_buffer_rsrc_t ys =
        __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
    const int cmin = p.half, cmax = kFft32L - p.half;
    const int64_t off = n0 - cmin - p.start;
    const int64_t oend = p.end - p.start;
    float pk = 0.0f;
    auto F = [&](int n, float &f0, float &f1) {
        const int s = (n & 1) ? sg : 0;
        f0 = __int_as_float(__float_as_int((float)o[n].x) ^ s);
        f1 = __int_as_float(__float_as_int((float)(-o[n].y)) ^ s);
    };
    if (r32_pair_path(p, n0, B)) {
        // pair stores: lane j's (c, c + 1) = 2 (j + 512 n) + {0, 1} as one 8-byte
        // store through a resource over exactly the unit's valid outputs
        // [n0, min(n0 + B, end)): the hardware range check drops the halo
        // (c < cmin wraps to a huge offset, c >= cmax lands past the end) and
        // the peak takes the lanes the same unsigned compare admits (whole
        // pairs: cmin and the record count are even)
        const int nrec = 4 * (int)(p.end - n0 < B ? p.end - n0 : B);
        const __amdgpu_buffer_rsrc_t yu =
            __builtin_amdgcn_make_buffer_rsrc(yb + (n0 - p.start), (short)0, nrec, 0x00020000);
        const int v0 = 8 * j - 4 * cmin;
        using b64_t = decltype(__builtin_amdgcn_raw_buffer_load_b64(yu, 0, 0, 0));
        static_assert(kR32PairStores == 32, "one pair store per register: the count the next unit's wait assumes");
#pragma unroll
        for (int n = 0; n < kR32PairStores; ++n) {
            float f0, f1;
            F(n, f0, f1);
            const int vo = v0 + 4096 * n;
            const float m = fmaxf(fabsf(f0), fabsf(f1));
            pk = (unsigned)vo < (unsigned)nrec ? fmaxf(pk, m) : pk;
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(b64_t, make_int2(__float_as_int(f0), __float_as_int(f1))), yu, vo, 0,
                kFft32StoreAux);
        }
    } else {
#pragma unroll
        for (int n = 0; n < 32; ++n) {
            const int c = 2 * (j + 512 * n);
            float f0, f1;
            F(n, f0, f1);
            const int64_t oo = off + c;
            const bool ok0 = c >= cmin && c < cmax && oo >= 0 && oo < oend,
                       ok1 = c + 1 >= cmin && c + 1 < cmax && oo + 1 >= 0 && oo + 1 < oend;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(oo * 4) : (int)0x80000000, 0,
                                                  kFft32StoreAux);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ok1 ? (int)(oo * 4 + 4) : (int)0x80000000,
                                                  0, kFft32StoreAux);
            pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
        }
    }
    return pk;
}

// fft_peak_stage with the wave's slot addressed from its wave-uniform index:
// the per-lane address fft_peak_stage derives from threadIdx.x was hoisted out
// of the unit loop and spilled (the kernel's only scratch access, a
// vector-memory reload on the path between the split DMA and the next unit's
// vmcnt(kR32PairStores))
__device__ __forceinline__ void r32_peak_stage(float *pk_lds, float pk) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) pk = fmaxf(pk, __shfl_xor(pk, s, 64));
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if ((threadIdx.x & 63) == 0) pk_lds[wv] = pk;
}

// The kernel's workgroup barriers order LDS only: __syncthreads()'s release
// fence would also wait for the wave's global stores (the previous unit's
// outputs, a fused normalize slice), which no other wave reads.
__device__ __forceinline__ void r32_bar() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Persistent, XCD-aware grid as fir_fft_f64_kernel (one 512-thread workgroup
// per CU, fft_unit32), zero-phase single-partition filters (kFftOutSym).
// pair: kR32PairTable (fft_plan_tables); tw: kR32Tw twiddles; task: 512
// r32_task_word; c8: the special lane's bin-N/2 coefficient (real).
// kNrm: the launch also rescales a previous file's outputs (FftNrm, as
// fir_fft_f64_kernel): unit u's slice is two halves, 2u and 2u + 1 of slice / 2
// floats, which the older waves (0..3) load, rescale and store one after the
// other while they wait at T1 backwards' first barrier (the younger waves
// arrive there thousands of cycles later).  Not at T1's first barrier: there
// the younger waves are still in the previous unit's memory phase, and a half
// moved there costs the config-5 step 2-3 % (scripts/variants/nrm_bar1.patch).
// Probe: phase-boundary hook (R32NoProbe in the product).
template <int kOut = kFftOutSym, bool kNrm = false, class Probe = R32NoProbe> // templates: host-only users emit no kernel stub
__global__ __launch_bounds__(kFftNT) void fir_fft32r_kernel(DirectParams p, const double2 *__restrict__ pair,
                                                           const double2 *__restrict__ tw,
                                                           const uint32_t *__restrict__ task, int B, FftGrid gd,
                                                           double c8, FftNrm nrm) {
    extern __shared__ double2 flds[];
    // the pair table's second half entry by entry (-2 %); the fused-rescale
    // kernel keeps the block load (the early loads spill 6 more VGPRs there)
    constexpr bool kPair2 = !kNrm;
    bool nrm_on = false;
    double nrm_gain = 1.0;
    if constexpr (kNrm) {
        float pkv = 0.0f;
        for (int i = 0; i < nrm.npeak; ++i) pkv = fmaxf(pkv, __uint_as_float(nrm.peak[i]));
        nrm_on = (pkv > 1.0f || nrm.force) && pkv > 0.0f;
        nrm_gain = 1.0 / (double)pkv;
        __builtin_amdgcn_s_setprio(1); // the older waves drop to 0 for their slices
    }
    // half h of unit u's normalize slice, by the older waves, at priority 0
    auto nrm_half = [&](int u, int h, int j, int wu) {
        if constexpr (kNrm) {
            if (nrm_on && wu < 4) {
                __builtin_amdgcn_s_setprio(0);
                FftNrm nh = nrm;
                nh.slice = nrm.slice / 2;
                float4 nv[kNrmK32];
                fft_nrm_load<kNrmK32>(nh, 2 * u + h, j, true, nv);
                fft_nrm_store<kNrmK32>(nh, 2 * u + h, j, nrm_gain, nv);
                __builtin_amdgcn_s_setprio(1);
            }
        }
    };
    double2 *twl = flds + kR32Work; // kR32Tw twiddles, then 8 f32 peak slots, then the special lane's scratch
    for (int i = threadIdx.x; i < kR32Tw; i += kFftNT) twl[i] = tw[i];
    float *pk_lds = reinterpret_cast<float *>(twl + kR32Tw);
    double2 *spl = twl + kR32Tw + 2;
    {
        const int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units);
        const int c = fft_div(u, gd);
        r32_stage_samples(p, c, p.seg0 + (int64_t)(u - c * gd.nseg) * B, threadIdx.x, flds);
    }
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    uint32_t tk_all = task[threadIdx.x];
    asm volatile("" : "+v"(tk_all));
    float pk_run = 0.0f;
    int pk_ch = -1;
    int pk_pending = -1;
    int rnd = 0;
    for (int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units); u < gd.units;
         u = fft_unit32(++rnd, blockIdx.x, gridDim.x, gd.units)) {
        int j = threadIdx.x;
        asm volatile("" : "+v"(j));
        const int w = j >> 6, lane = j & 63;
        const int wu = __builtin_amdgcn_readfirstlane(w);
        const bool hi = wu >= 4; // waves 4..7: rotated stage-1 / final DFT32s
        const int ch = fft_div(u, gd);
        const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;
        double2 a[32];
        // the staging transfers have landed; the previous unit's pair stores
        // (issued after them) may still be in flight.  The older waves issued
        // the younger waves' transfers too: everyone waits for their waits.
        __builtin_amdgcn_s_waitcnt(r32_vmcnt(kR32PairStores));
        r32_bar();
        Probe::stamp(0, rnd);
        // ---- stage 1: the samples out of the wave's region (staged by the
        // previous unit), waves 4..7 negating the odd ones; DFT32; W_16384^(b k1)
        {
            const float2 *fz = reinterpret_cast<const float2 *>(flds) + 2 * kR32Rg * w + lane;
            const int sg = hi ? (int)0x80000000 : 0;
#pragma unroll
            for (int n = 0; n < 32; ++n) {
                float2 vn = fz[64 * n];
                if (n & 1) {
                    vn.x = __int_as_float(__float_as_int(vn.x) ^ sg);
                    vn.y = __int_as_float(__float_as_int(vn.y) ^ sg);
                }
                a[n] = make_double2((double)vn.x, (double)vn.y);
            }
        }
        dft32(a);
        {
            // register r holds k1 = r + 16 hi (mod 32): powers w^(16 hi) w^r, w^(16 (1 - hi)) w^(r - 16)
            const double2 wb = twl[kR32TwB + j], w16 = twl[kR32TwB16 + j];
            r32_chain_k1acc(a, wb, w16, hi);
        }
        Probe::stamp(1, rnd);
        // ---- T1 round 1: registers 0..15 into the wave's own region (its lanes
        // read their samples from it above: issue order is enough)
#pragma unroll
        for (int i = 0; i < 16; ++i) flds[kR32Rg * w + 64 * i + lane] = a[i];
        Probe::stamp(2, rnd);
        r32_bar();
        Probe::stamp(3, rnd);
        if (pk_pending >= 0) {
            if (threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
            pk_pending = -1;
        }
        const int g = lane >> 5, h = (lane >> 4) & 1, gam = lane & 15;
        const int k1 = r32_column(w, g, h);
        double2 c[32];
        {
            // from thread b = 16 (i + 16 h) + gam, its register k1 & 15
            const int base = 4 * kR32Rg * h + 64 * (k1 & 15) + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) c[i] = flds[base + kR32Rg * (i >> 2) + 16 * (i & 3)];
        }
        Probe::stamp(4, rnd);
        r32_bar();
        Probe::stamp(5, rnd);
        // ---- T1 round 2: registers 16..31 (k1 = 16 + i, or i for waves 4..7)
        // into the region of their column's wave
        {
            const int base = 16 * ((j >> 4) & 15) + (j & 15);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int home = hi ? r32_column_home(i) : r32_column_home(16 + i); // uniform
                flds[kR32Rg * (home >> 2) + 256 * (home & 3) + base] = a[16 + i];
            }
        }
        Probe::stamp(6, rnd);
        r32_bar();
        {
            const int base = kR32Rg * w + 256 * (2 * g + h) + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) c[16 + i] = flds[base + 16 * i];
        }
        Probe::stamp(7, rnd);
        // ---- stage 2: DFT32 over beta (rotated by 16 h), * (s W_512^gam)^kappa, s = (-1)^h
        double2 pq[16], p2v[8];
        dft32(c);
        double2 wg = twl[kR32TwG + gam];
        if (h) wg = make_double2(-wg.x, -wg.y);
        r32_chain32acc(c, wg);
        Probe::stamp(8, rnd);
        // ---- the pair table's first half, in flight across T2
        {
            const double2 *pt = pair + j;
#pragma unroll
            for (int i = 0; i < 8; ++i) pq[i] = pt[512 * i];
#pragma unroll
            for (int m = 0; m < 4; ++m) p2v[m] = pt[512 * (16 + m)];
        }
        __builtin_amdgcn_sched_barrier(0);
        Probe::stamp(9, rnd);
        // ---- T2: two wave-local rounds (kappa < 16, kappa >= 16) in the wave's region
        uint32_t tk = tk_all;
        asm volatile("" : "+v"(tk)); // per unit: T2's addresses are not hoisted out of the loop
        const int x1 = (tk >> 1) & 15, x2 = (tk >> 6) & 15;
        const int rb1 = kR32Rg * w + kR32Gs * g + kR32Hs * (tk & 1) + kR32Row * x1;
        const int rb2 = kR32Rg * w + kR32Gs * g + kR32Hs * ((tk >> 5) & 1) + kR32Row * x2;
        const int wb2 = kR32Rg * w + kR32Gs * g + kR32Hs * h;
        double2 R1[16], R2[16];
#pragma unroll
        for (int kl = 0; kl < 16; ++kl) flds[r32_t2(wb2, kl, gam)] = c[kl];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) R1[i] = flds[r32_t2r(rb1, i)];
        wave_lds_sync();
#pragma unroll
        for (int kl = 0; kl < 16; ++kl) flds[r32_t2(wb2, kl, gam)] = c[16 + kl];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) R2[i] = flds[r32_t2r(rb2, i)];
        Probe::stamp(10, rnd);
        // ---- stage 3: DFT16 over gamma -> lambda
        dft16f(R1);
        dft16f(R2);
        Probe::stamp(11, rnd);
        // ---- pair step: slot i pairs R1[i] (bin k) with R2[15 - i] (bin N - k);
        // the special lane permutes its registers into that layout first
        const bool sp = wu == 0 && lane == kR32SpecialLane;
        double2 v8 = R1[8];
        if (wu == 0) {
            if (sp) {
                // x' = [R2 0..7, R1 1..7, R1 0], y' = [R1 0, R1 9..15, R2 8..15]; R1[8] (bin N/2) apart
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    spl[i] = R1[i];
                    spl[16 + i] = R2[i];
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) R1[i] = spl[16 + i];
#pragma unroll
                for (int i = 8; i < 15; ++i) R1[i] = spl[i - 7];
                R1[15] = spl[0];
                R2[0] = spl[0];
#pragma unroll
                for (int i = 1; i < 8; ++i) R2[i] = spl[8 + i];
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            fft_pair_sym(R1[i], R2[15 - i], pq[i].x, pq[i].y, (i & 1) ? p2v[i >> 1].y : p2v[i >> 1].x, R1[i],
                         R2[15 - i]);
            if constexpr (kPair2) {
                // the second half's entry 8 + i into the registers pair i has
                // just freed, so each load has the remaining pairs to land in
                pq[8 + i] = pair[j + 512 * (8 + i)];
                if (i & 1) p2v[4 + (i >> 1)] = pair[j + 512 * (20 + (i >> 1))];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (!kPair2) {
            // the second half of the table (its registers were the first half's)
            const double2 *pt = pair + j;
#pragma unroll
            for (int i = 8; i < 16; ++i) pq[i] = pt[512 * i];
#pragma unroll
            for (int m = 4; m < 8; ++m) p2v[m] = pt[512 * (16 + m)];
        }
#pragma unroll
        for (int i = 8; i < 16; ++i) {
            fft_pair_sym(R1[i], R2[15 - i], pq[i].x, pq[i].y, (i & 1) ? p2v[i >> 1].y : p2v[i >> 1].x, R1[i],
                         R2[15 - i]);
            __builtin_amdgcn_sched_barrier(0);
        }
        Probe::stamp(12, rnd);
        if (wu == 0) {
            if (sp) {
                // back: R1 = [x 15, x 8..14, conj(c8 v8), y 1..7], R2 = [x 0..7, y 8..15]
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    spl[i] = R1[i];
                    spl[16 + i] = R2[i];
                }
                R1[0] = spl[15];
#pragma unroll
                for (int i = 1; i < 8; ++i) R1[i] = spl[7 + i];
                R1[8] = make_double2(v8.x * c8, -v8.y * c8);
#pragma unroll
                for (int i = 9; i < 16; ++i) R1[i] = spl[16 + i - 8];
#pragma unroll
                for (int i = 0; i < 8; ++i) R2[i] = spl[i];
            }
        }
        // ---- inverse stage 3: DFT16 over lambda -> gamma (on conj(V))
        dft16f(R1);
        dft16f(R2);
        Probe::stamp(13, rnd);
        // ---- T2 backwards (addresses recomputed from laundered words: the 32
        // of T2 would otherwise stay live across the pair step)
        {
            uint32_t tkb = tk_all;
            int jb = threadIdx.x;
            asm volatile("" : "+v"(tkb), "+v"(jb));
            const int wb_ = jb >> 6, gb_ = (jb >> 5) & 1, hb_ = (jb >> 4) & 1, gmb = jb & 15;
            const int y1 = (tkb >> 1) & 15, y2 = (tkb >> 6) & 15;
            const int sb1 = kR32Rg * wb_ + kR32Gs * gb_ + kR32Hs * (tkb & 1) + kR32Row * y1;
            const int sb2 = kR32Rg * wb_ + kR32Gs * gb_ + kR32Hs * ((tkb >> 5) & 1) + kR32Row * y2;
            const int sbw = kR32Rg * wb_ + kR32Gs * gb_ + kR32Hs * hb_;
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[r32_t2r(sb1, i)] = R1[i];
            wave_lds_sync();
#pragma unroll
            for (int kl = 0; kl < 16; ++kl) c[kl] = flds[r32_t2(sbw, kl, gmb)];
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[r32_t2r(sb2, i)] = R2[i];
            wave_lds_sync();
#pragma unroll
            for (int kl = 0; kl < 16; ++kl) c[16 + kl] = flds[r32_t2(sbw, kl, gmb)];
        }
        Probe::stamp(14, rnd);
        // ---- inverse stage 2: * (s W_512^gam)^kappa, DFT32 (outputs rotated by 16 h).
        // The powers are rebuilt, not kept from stage 2 (124 VGPRs across the
        // pair step): the laundered base stops the compiler from reusing them.
        asm volatile("" : "+v"(wg.x), "+v"(wg.y));
        r32_chain32acc(c, wg);
        dft32(c);
        wave_lds_sync();
        Probe::stamp(15, rnd);
        // ---- T1 backwards, round 1: registers 0..15 into the wave's own region
#pragma unroll
        for (int i = 0; i < 16; ++i) flds[kR32Rg * w + 64 * i + lane] = c[i];
        Probe::stamp(16, rnd);
        nrm_half(u, 0, j, wu);
        nrm_half(u, 1, j, wu);
        r32_bar();
        Probe::stamp(17, rnd);
        {
            // thread b: register r holds k1 = r + 16 hi, from lane (k1, gamma_b)'s register beta_b & 15
            const int base = 64 * ((j >> 4) & 15) + (j & 15);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int home = hi ? r32_column_home(16 + r) : r32_column_home(r); // uniform
                a[r] = flds[kR32Rg * (home >> 2) + 16 * (home & 3) + base];
            }
        }
        Probe::stamp(18, rnd);
        r32_bar();
        Probe::stamp(19, rnd);
        {
            // registers 16..31: beta = i + 16 (1 - h) -> thread 16 beta + gam's region
            const int base = 4 * kR32Rg * (1 - h) + 64 * (k1 & 15) + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[base + kR32Rg * (i >> 2) + 16 * (i & 3)] = c[16 + i];
        }
        Probe::stamp(20, rnd);
        r32_bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) a[16 + i] = flds[kR32Rg * w + 64 * i + lane];
        Probe::stamp(21, rnd);
        // vmcnt(0) lgkmcnt(0): the wave's reads of its region have retired (and
        // the compiler's vmcnt accounting ignores LDS-DMA; see fir_fft32.hpp)
        {
            __builtin_amdgcn_s_waitcnt(0x0070);
            r32_bar(); // every wave's reads of its region have returned
            const int un1 = fft_unit32(rnd + 1, blockIdx.x, gridDim.x, gd.units);
            const int un = un1 < gd.units ? un1 : u;
            const int cn = fft_div(un, gd);
            const int64_t nn = p.seg0 + (int64_t)(un - cn * gd.nseg) * B;
            const bool split = r32_interior(p, nn);
            if (!split) r32_stage_samples(p, cn, nn, j, flds);
            Probe::stamp(22, rnd);
            // ---- final: * W_16384^(b k1), DFT32 over k1 -> n (an interior next
            // unit's DMA issued in quarters between the VALU blocks, so a wave
            // whose transfer waits for the CU's memory queue still computes).
            // The older waves (0..3) issue every region's transfers, theirs and
            // wave + 4's: the younger waves, which leave the final phase last
            // (their VALU issues second), then only compute and store
            // (config 2 launch -6 %, config 4 -5 %, scripts/variants/README.md)
            auto part = [&](auto q) {
                constexpr int k = decltype(q)::value;
                if (split && !hi) {
                    __builtin_amdgcn_sched_barrier(0);
                    r32_dma_part<4 * k, 4 * k + 4>(p, cn, nn, j, flds);
                    r32_dma_part<4 * k, 4 * k + 4>(p, cn, nn, j + 256, flds);
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            const double2 wb = twl[kR32TwB + j], w16 = twl[kR32TwB16 + j], one = make_double2(1.0, 0.0);
            part(std::integral_constant<int, 0>{});
            {
                const double2 w2 = cmul(wb, wb);
                const double2 w4 = cmul(w2, w2);
                r32_chain_anchored<16>(a, 0, csel(hi, w16, one), wb, w4);
                part(std::integral_constant<int, 1>{});
                r32_chain_anchored<16>(a, 16, csel(hi, one, w16), wb, w4);
            }
            part(std::integral_constant<int, 2>{});
            dft32_hook(a, [&] { part(std::integral_constant<int, 3>{}); });
        }
        // pair-path units: the DMA wait moves to the next unit's top (its
        // vmcnt(kR32PairStores) lets exactly these stores stay in flight);
        // the other units wait for the staging transfers here
        if (!r32_pair_path(p, n0, B)) __builtin_amdgcn_s_waitcnt(kVmcnt0);
        const float pk = r32_store_unit(p, ch, n0, B, j, a, hi ? (int)0x80000000 : 0);
        if (ch != pk_ch) {
            if (p.peak && pk_ch >= 0) {
                r32_peak_stage(pk_lds, pk_run);
                pk_pending = pk_ch;
                asm volatile("" : "+v"(pk_pending));
            }
            pk_run = 0.0f;
            pk_ch = ch;
        }
        pk_run = fmaxf(pk_run, pk);
        Probe::stamp(23, rnd);
    }
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    if (p.peak && pk_ch >= 0) {
        __syncthreads();
        if (pk_pending >= 0 && threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
        __syncthreads();
        fft_peak_stage(pk_lds, pk_run);
        __syncthreads();
        if (threadIdx.x == 0) fft_peak_commit(p, pk_ch, pk_lds);
    }
}

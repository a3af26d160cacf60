// fir_fft.hpp -- f64 overlap-save FFT evaluation of the FilterCore.h hot path.
//
// Same contract as fir_direct.hpp (y[n] = sum_k h[k] x[n - half + k], zero
// padding outside [0,N), outputs [start,end), RNE to f32), evaluated with
// f64 FFTs instead of T multiply-adds per sample.
//
// One unit = one segment of B = L - T + 1 consecutive outputs:
//   x_seg[i] = x[n0 - half + i], i in [0, L), L = 16384 real samples
//   c = IFFT_L( FFT_L(x_seg) * G ),  G = FFT_L(reversed taps, zero padded)
//   y[n0 + m - (T-1)] = c[m] for m in [T-1, L)          (overlap-save)
// A linear-phase (symmetric) filter runs in zero-phase form instead
// (kFftOutSym): G = FFT_L of the taps centred on sample 0 is real, the pair
// table is real, and y[n0 + m - half] = c[m] for m in [half, L - half).
// The real length-L transform is one complex M = L/2 = 8192-point FFT of
// z[m] = x_seg[2m] + i x_seg[2m+1]; the even/odd split and merge are fused
// with the multiply by G into one "pair" step on bins k and M-k; the inverse
// is conj(FFT(conj(V))).  All scale factors live in the pair table.
//
// Four-step decomposition, M = 16 x 512 (index flow, lane
// tables and LDS bank patterns are checked by scripts/fft_lds_sim.py):
//   stage 1 (thread b of 512): 16-point DFT over z[512 a + b] -> column c,
//           times W_8192^(b c); one workgroup-wide transpose into LDS column
//           blocks [c][b];
//   wave w owns the two columns {w, 16-w} (wave 0: {0, 8}) and does their
//           512-point DFTs as 8 x 8 x 8 with two wave-local LDS exchanges --
//           no workgroup barrier;
//   the lane assignment of the last exchange is mirrored between a wave's two
//           columns, so bins k and M-k sit in the same lane: the pair step runs
//           in registers (wave 0 needs one lane, kFftSpecialLane, permuted);
//   the inverse runs the same stages in transposed order and ends with one
//           workgroup-wide transpose and the 16-point DFTs.
// Per segment: 2 workgroup barriers and 6 LDS round trips of the 128 KiB work
// array (the radix-16x16x16x2 Stockham form it replaces needed 14 barriers and
// ~8 round trips).  The grid is persistent (one 512-thread workgroup per CU)
// and XCD-aware (fft_unit: neighbouring segments on one XCD share their halo
// in its L2); samples are read and results written (non-temporal) through
// range-checked raw buffer resources, so the channel-edge zero padding and
// output clipping need no branches.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "fir_direct.hpp"

// Phase timestamps for tools/fft_trace.hip (off in the product build): lane 0
// of every wave of workgroups < 64 records s_memtime at each phase boundary of
// its 5th unit (round 4).
#ifdef LCFIR_FFT_TRACE
__device__ unsigned long long g_fft_trace[64][8][24];
#define FFT_STAMP(i)                                                                     \
    do {                                                                                 \
        if (blockIdx.x < 64 && rnd == 4 && (threadIdx.x & 63) == 0)                      \
            g_fft_trace[blockIdx.x][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define FFT_STAMP(i) \
    do {             \
    } while (0)
#endif

// Per-unit timeline for tools/launch_trace.hip (off in the product build):
// thread 0 of every workgroup records s_memrealtime (100 MHz, chip-wide) at
// kernel entry (slot 0), at the top of each unit (slots 1..) and at exit.
#ifdef LCFIR_FFT_UTRACE
constexpr int kUtraceSlots = 160;
__device__ unsigned long long g_fft_utrace[1024][kUtraceSlots];
__device__ unsigned long long g_fft_uclock[1024][2]; // s_memtime (shader clock) at entry, exit
#define FFT_USTAMP(slot)                                                                    \
    do {                                                                                    \
        if (threadIdx.x == 0 && blockIdx.x < 1024) {                                        \
            g_fft_utrace[blockIdx.x][min((int)(slot), kUtraceSlots - 1)] =                  \
                __builtin_amdgcn_s_memrealtime();                                           \
            g_fft_uclock[blockIdx.x][(slot) == 0 ? 0 : 1] = __builtin_amdgcn_s_memtime();   \
        }                                                                                   \
    } while (0)
#else
#define FFT_USTAMP(slot) \
    do {                 \
    } while (0)
#endif


namespace lcfir {

constexpr int kFftL = 16384;        // real segment length
constexpr int kFftM = kFftL / 2;    // complex FFT length
constexpr int kFftNT = 512;         // threads per workgroup
constexpr int kFftMinB = 2048;      // smallest useful segment (B = L - T + 1)
constexpr int kFftTw = 512 + 64;    // LDS twiddles: W_8192^i (i < 512), W_512^i (i < 64)
constexpr int kFftMaxPartTaps = kFftL - kFftMinB + 1; // longest partition (14 337 taps)
constexpr int kFftPairSlots = 9;    // pair-table slots per thread (8 pairs + k = M/2)
constexpr int kFftSpecialLane = 35; // wave-0 lane holding the self-paired bins 0 and M/2
constexpr int kVmcnt0 = 0x0F70;     // s_waitcnt vmcnt(0) (expcnt, lgkmcnt left at their maxima)
// cache policy of the f32 output stores: nt (non-temporal).  The outputs are
// written once and every workgroup stores its segment in the same phase; nt
// stores drain that burst faster (+5 % on config 2; nt, sc0 or sc1 on the
// sample loads measured 0 to -5 %, so those stay cached)
constexpr int kNtStore = 2;
// output modes of fir_fft_f64_kernel (see there)
constexpr int kFftOutF32 = 0, kFftOutFirst = 1, kFftOutAdd = 2, kFftOutLast = 3, kFftOutSym = 4;
// kFftOutSym = kFftOutF32 for a linear-phase filter in zero-phase form: real
// pair table (fft_plan_build's symmetric layout), outputs c in [half, L - half)
// zero-phase table: double2 (p1, q2) per (slot, thread), then double2 (p2 of
// slot 2m, p2 of slot 2m+1) per (m, thread) -- fft_pair_sym's coefficients,
// computed on the host in long double (fft_plan_build)
constexpr int kFftSymPQ = 0, kFftSymP2 = 8 * kFftNT;

// Wave 0, lanes 32..63: the column-0 task pairs (d1A | e1A << 3 | d1B << 6 |
// e1B << 9), ordered so the exchange-2 reads and exchange-3 writes stay
// bank-conflict free (generated and checked by scripts/fft_lds_sim.py).
constexpr uint16_t kFftWave0C0[32] = {
    0xf43, 0x99a, 0xfc1, 0x020, 0x4ed, 0xe47, 0xc8e, 0xb14, 0x89e, 0xec5, 0x85f,
    0xd0c, 0x373, 0x3f1, 0xc10, 0x5aa, 0xb92, 0x91c, 0xe86, 0xad5, 0xa18, 0x95b,
    0x5e9, 0x46f, 0xf82, 0xe08, 0x8dd, 0x2b6, 0xf04, 0xd4b, 0x9d9, 0x277};

constexpr int kFftMaxTaps = 1 << 20; // longest filter (partitions of <= kFftMaxPartTaps)
constexpr size_t kFftPairTable = (size_t)3 * kFftPairSlots * kFftNT; // double2 per pair table

// Per-context choices of the FFT method (lcfir_ctx_set_fft_tuning, include/lcfir.h).
// The defaults are the product's; tests set the others explicitly (no
// environment variable is read anywhere in the library).
struct FftTuning {
    int32_t seg_len = 0;    // segment length in real samples: 0 = by tap count (fft_choose_seg_len), 16384, 32768
    int32_t zero_phase = 1; // 1: linear-phase filters run in zero-phase form (fft_sym_eligible); 0: general table
    int64_t chunk = 0;      // outputs per launch chunk; 0 = 2^28 (the buffer offsets' 32-bit range)
    int64_t max_units = 0;  // units per launch; 0 = 2^31 - 1 (FftGrid's 32-bit unit index)
    // kernel family of zero-phase single-partition plans (lcfir_ctx_set_fft_family):
    // kFamilyDefault or kFamilyLds (the LDS-column kernels everywhere)
    int32_t family = 0;
};

// A filter longer than one segment allows is split into `parts` equal
// partitions of `ntaps` taps (odd, zero padded at the end), each convolved by
// its own launch with the input offset half - p * ntaps; the launches sum in
// f64 (fir_fft_f64_kernel's output modes).
struct FftPlan {
    bool ready = false;
    int L = 16384;             // segment length (real samples): fir_fft_f64_kernel or, 32768, fir_fft32_f64_kernel
    int ntaps = 0;             // taps per partition (the filter's own count when parts == 1)
    int parts = 1;
    int B = 0;                 // outputs per segment = L - ntaps + 1
    double2 *d_pair = nullptr; // parts x halves x [3][kFftPairSlots][512]: 2S, 2D, W_L^k per (slot, thread)
    std::vector<double2> c8;   // per partition: the special lane's bin-M/2 coefficient
    double2 *d_tw = nullptr;   // kFftTw twiddles (kFft32Tw for L = 32768)
    uint32_t *d_task = nullptr; // [halves][512] task words (cA, d1A, e1A, cB, d1B, e1B)
    int cus = 256;             // compute units of the plan's device (persistent grid)
    bool sym = false;          // linear-phase filter run in zero-phase form (kFftOutSym)
    bool reg32 = false;        // L = 32768 zero-phase on the register-resident kernel (fir_fft32r.hpp)
    FftTuning tune;            // the ctx's tuning when the plan was built
};

// A filter runs in zero-phase form (kFftOutSym: real pair table, a cheaper
// pair step) when it is one partition and it is symmetric, h[k] = h[T-1-k], up to an
// antisymmetric part of at most 2^-50 of its l1 norm.  Dropping that part
// changes any output by at most 2^-50 |h|_1 max|x| -- the size of the f64
// FFT's own rounding error.  FftTuning::zero_phase = 0 turns the form off.
inline bool fft_sym_eligible(const std::vector<double> &h, int parts, const FftTuning &tune) {
    const int T = (int)h.size();
    if (!tune.zero_phase || parts != 1 || T < 3) return false;
    long double anti = 0.0L, norm = 0.0L;
    for (int k = 0; k < T; ++k) {
        anti += fabsl(((long double)h[(size_t)k] - (long double)h[(size_t)(T - 1 - k)]) * 0.5L);
        norm += fabsl((long double)h[(size_t)k]);
    }
    return norm > 0.0L && anti <= norm * 0x1p-50L;
}

inline bool fft_supported(int ntaps) { return ntaps >= 1 && ntaps <= kFftMaxTaps; }
// AUTO's choice: the direct kernel (bit-exact, strict fma order) up to 63
// taps, where it is as fast as the FFT or faster (config-2 shape, r03:
// 658 / 562 / 451 / 375 Gs/s at 15 / 31 / 47 / 63 taps vs the FFT's flat
// ~360), the FFT above (365 vs 317 at 79 taps, 364 vs 275 at 95)
inline bool fft_preferred(int ntaps) { return ntaps >= 64 && fft_supported(ntaps); }

// taps per partition when `parts` partitions share `ntaps` taps (odd: the
// kernel's output pairing assumes an even T - 1)
inline int fft_partition_taps(int ntaps, int parts) {
    const int t = (ntaps + parts - 1) / parts;
    return t | 1;
}
// partition count minimising the work per output, parts / (L - taps + 1), for
// segments of L real samples (a partition keeps at least kFftMinB outputs)
inline int fft_partition_count(int ntaps, int L = 16384) {
    int best = 0;
    double best_cost = 0.0;
    for (int n = 1; n <= ntaps; ++n) {
        const int t = fft_partition_taps(ntaps, n);
        if (t > L - kFftMinB + 1) continue;
        const double cost = (double)n / (double)(L - t + 1);
        if (best == 0 || cost < best_cost) {
            best = n;
            best_cost = cost;
        }
        if (t < L / 4) break; // more partitions only add launches from here
    }
    return best;
}
// Time of one unit relative to a single-partition L = 16 384 unit, measured
// on MI355X with tools/fft32_trace.hip (config-3 shape, 6 001 .. 30 001 taps,
// CHANGELOG.md s4.2): a partitioned L = 16 384 pass also reads and writes its f64
// partial sums; an L = 32 768 unit is two 8192-point halves plus the split,
// the merge and the park slab, the general pair table and partitions cost
// more there (register pressure).
// Zero-phase single-partition L = 32768 plans run fir_fft32r_kernel (the
// transform held in registers); its unit costs 2.2 L = 16 384 units (configs 2 and 3: 23.6 us against 10.7 us per
// persistent-grid round, CHANGELOG.md s4.2), so it takes linear-phase filters
// from ~4 000 taps (config 2's 4 001: 7.65e-5 against 8.07e-5 per output).
constexpr double kFft32rUnitCost = 2.2;
// FftTuning::family: the default takes fir_fft32r at L = 32 768 and the
// LDS-column kernel at L = 16 384; kFamilyLds the LDS-column kernels at both.
// (Family 2, round 5's L = 16 384 two-workgroups-per-CU register kernel, is a
// variant patch now: scripts/variants/r16_kernel.patch, not faster on any
// config.)
constexpr int kFamilyDefault = 0, kFamilyLds = 1;
inline bool fft_reg32(int L, int parts, bool sym, const FftTuning &tune = FftTuning{}) {
    return L == 32768 && parts == 1 && sym && tune.family != kFamilyLds;
}
inline double fft_unit_cost(int L, int parts, bool sym, const FftTuning &tune = FftTuning{}) {
    if (L == 16384) return parts == 1 ? 1.0 : 1.25;
    if (fft_reg32(L, parts, sym, tune)) return kFft32rUnitCost;
    return parts == 1 ? (sym ? 2.9 : 3.1) : 4.0;
}
// Estimated time per output with segment length L: partitions x unit cost /
// outputs per segment.  Infinity when L cannot hold the filter.
inline double fft_seg_estimate(const std::vector<double> &h, int L, const FftTuning &tune) {
    const int ntaps = (int)h.size();
    const int parts = fft_partition_count(ntaps, L);
    if (parts == 0) return 1e300;
    const int B = L - (parts == 1 ? ntaps : fft_partition_taps(ntaps, parts)) + 1;
    return fft_unit_cost(L, parts, fft_sym_eligible(h, parts, tune), tune) * parts / (double)B;
}
// Segment length for a filter (FftTuning::seg_len = 0): the lower cost per
// output, the longer segment only when it saves at least 5 %.  A function of
// the taps and the tuning alone, never of a call's shape: the segment grid
// must not change under a ctx (partition invariance, fft_grid_start), and
// every entry point (range, window, channels, fft_info), every --devices
// stage and every rank then builds the same plan for the same filter, so a
// file's bytes do not depend on which call came first.  Long
// filters take L = 32 768 (one partition up to 30 721 taps instead of two
// from 10 900, 2x faster at 12 001 .. 19 201 taps); config 1's 48 000-sample
// launch at 19 201 taps measured equal either way (0.0386 vs 0.0387 ms, the
// graph-replayed step 3 % faster with 32 768, CHANGELOG.md s0).
inline int fft_choose_seg_len(const std::vector<double> &h, const FftTuning &tune) {
    return fft_seg_estimate(h, 32768, tune) < 0.95 * fft_seg_estimate(h, 16384, tune) ? 32768 : 16384;
}

// LDS slot of column c: a wave's two columns sit in adjacent 8 KiB blocks
// (w -> 2w, 16-w -> 2w+1; wave 0: 0 -> 0, 8 -> 1), so its second column's
// exchange addresses are the first's plus an immediate offset.
__host__ __device__ constexpr int fft_slot(int c) {
    return c == 0 ? 0 : c == 8 ? 1 : c < 8 ? 2 * c : 33 - 2 * c;
}
constexpr int fft_slot_column(int s) { return s == 0 ? 0 : s == 1 ? 8 : s % 2 == 0 ? s / 2 : (33 - s) / 2; }

// Unit processed by workgroup b in round i of a persistent grid of g
// workgroups.  Workgroups are dealt to the 8 XCDs round-robin (b mod 8), so
// XCD x gets the g/8 consecutive units i g + x g/8 + (b div 8): a segment and
// its neighbour share the T-1 halo samples, and on one XCD the second read of
// the halo hits that XCD's L2 instead of HBM.  The last, partial round gives
// unit i g + b to workgroup b: its units spread over all 8 XCDs, and on each
// XCD they go to the workgroups dispatched first.  A launch queued behind
// this one on another stream fills the CUs the tail leaves idle; its own
// extra-unit workgroups then start early instead of behind the tail.  A
// bijection on every round, so the last round covers [i g, units) exactly.
__host__ __device__ inline int64_t fft_unit(int64_t i, int b, int g, int64_t units) {
    const int64_t base = i * g;
    if (g % 8 != 0 || base + g > units) return base + b;
    return base + (int64_t)(b % 8) * (g / 8) + b / 8;
}
// the same map in 32-bit arithmetic (fft_launch keeps every launch's units < 2^31)
__host__ __device__ inline int fft_unit32(int i, int b, int g, int units) {
    const int base = i * g;
    if (g % 8 != 0 || base + g > units) return base + b;
    return base + (b % 8) * (g / 8) + b / 8;
}

// A launch's unit grid: nch x nseg (channel, segment) units, units < 2^31.
// The kernels split a unit index into (channel, segment) with a multiply and
// a shift instead of a division: m = ceil(2^(31+l) / nseg), l = ceil(log2
// nseg), gives u / nseg = (u m) >> (31 + l) exactly for every u < 2^31 (the
// round-up method; m < 2^32).  The 64-bit division it replaces expanded to
// ~130 scalar instructions, twice per segment, and spilled SGPRs.
struct FftGrid {
    int32_t nseg;  // segments per channel
    int32_t units; // channels x nseg
    uint32_t m;    // ceil(2^(31+l) / nseg)
    uint32_t sh;   // 31 + l
};
inline FftGrid fft_grid(int64_t nseg, int64_t units) {
    FftGrid g{(int32_t)nseg, (int32_t)units, 0u, 31u};
    uint32_t l = 0;
    while (((int64_t)1 << l) < nseg) ++l;
    const uint64_t num = (uint64_t)1 << (31 + l);
    g.m = (uint32_t)((num + (uint64_t)nseg - 1) / (uint64_t)nseg);
    g.sh = 31 + l;
    return g;
}
__host__ __device__ inline int fft_div(int u, const FftGrid &g) {
    return (int)(((uint64_t)(uint32_t)u * g.m) >> g.sh);
}

// Task word of thread t = 64 w + lane after exchange 2: task A = (cA, d1A, e1A),
// task B = (cB, d1B, e1B); bins k = c + 16 (d1 + 8 e1 + 64 e2), e2 = register.
// Waves 1..7: columns w and 16 - w, B mirrors A, so X[k] (A[e2]) and X[M-k]
// (B[7-e2]) share a lane.  Wave 0: lanes 0..31 column-8 mirror pairs, lanes
// 32..63 column-0 partner pairs (kFftWave0C0).
inline uint32_t fft_task_word(int t) {
    const int w = t >> 6, lane = t & 63;
    int ca, da, ea, cb, db, eb;
    if (w != 0 || lane < 32) {
        ca = w ? w : 8;
        cb = w ? 16 - w : 8;
        da = lane & 7;
        ea = lane >> 3;
        db = 7 - da;
        eb = 7 - ea;
    } else {
        const int v = kFftWave0C0[lane - 32];
        ca = cb = 0;
        da = v & 7;
        ea = (v >> 3) & 7;
        db = (v >> 6) & 7;
        eb = (v >> 9) & 7;
    }
    // the column fields hold LDS slots (fft_slot): the kernel only addresses with them
    return (uint32_t)(fft_slot(ca) | da << 4 | ea << 7 | fft_slot(cb) << 10 | db << 14 | eb << 17);
}

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
// per-component select: a ternary on a double2 can be lowered through scratch
// memory (store both, load by a lane-dependent address)
__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
    return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}
__device__ __forceinline__ double2 mul_mi(double2 a) { return make_double2(a.y, -a.x); } // * (-i)
__device__ __forceinline__ double2 mul_pi(double2 a) { return make_double2(-a.y, a.x); } // * (+i)

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

// The W8^1 = (1-i)/sqrt2 and W8^3 = -(1+i)/sqrt2 rotations leave their sqrt(1/2)
// factor pending (u1 = sqrt2 a W8^1, u3 = sqrt2 a W8^3: adds only), and the
// butterfly that consumes them folds it into FMAs.
__device__ __forceinline__ double2 rot8_1(double2 a) { return make_double2(a.x + a.y, a.y - a.x); }
__device__ __forceinline__ double2 rot8_3(double2 a) { return make_double2(a.y - a.x, -(a.x + a.y)); }
// t0 + kR2 u, t0 - kR2 u
__device__ __forceinline__ void fma_pm(double2 t0, double2 u, double2 &p, double2 &m) {
    p = make_double2(__builtin_fma(kR2, u.x, t0.x), __builtin_fma(kR2, u.y, t0.y));
    m = make_double2(__builtin_fma(-kR2, u.x, t0.x), __builtin_fma(-kR2, u.y, t0.y));
}
// dft4(a0, a1, a2, a3) for a1 = kR2 u1, a3 = kR2 u3 (sqrt(1/2) pending on both odd inputs)
__device__ __forceinline__ void dft4_r13(double2 &a0, double2 u1, double2 &a2, double2 u3, double2 &o1,
                                         double2 &o3) {
    const double2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
    const double2 s = cadd(u1, u3), d = csub(u1, u3);
    // t2 = kR2 s, t3 = -i kR2 d
    fma_pm(t0, s, a0, a2);
    o1 = make_double2(__builtin_fma(kR2, d.y, t1.x), __builtin_fma(-kR2, d.x, t1.y));
    o3 = make_double2(__builtin_fma(-kR2, d.y, t1.x), __builtin_fma(kR2, d.x, t1.y));
}
// dft4(a0, a1, a2, a3) for a2 = kR2 u2 (sqrt(1/2) pending on input 2)
__device__ __forceinline__ void dft4_r2(double2 &a0, double2 &a1, double2 u2, double2 &a2, double2 &a3) {
    double2 t0, t1;
    fma_pm(a0, u2, t0, t1);
    const double2 t2 = cadd(a1, a3), t3 = mul_mi(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

constexpr double kT1 = 0.41421356237309504880; // tan(pi/8)
// W16^1, W16^3 and W16^9 are cos(pi/8) times (1 - i tan), -i (1 + i tan) and
// -(1 - i tan): the rotations by tan are two FMAs each (no MUL) and the common
// cos(pi/8) stays pending into the row's radix-4, whose last adds become FMAs.
__device__ __forceinline__ double2 rot16_1(double2 a) { // a W16^1 / kC1
    return make_double2(__builtin_fma(kT1, a.y, a.x), __builtin_fma(-kT1, a.x, a.y));
}
__device__ __forceinline__ double2 rot16_3(double2 a) { // a W16^3 / kC1
    return make_double2(__builtin_fma(kT1, a.x, a.y), __builtin_fma(kT1, a.y, -a.x));
}
__device__ __forceinline__ double2 rot16_9(double2 a) { // a W16^9 / kC1
    return make_double2(__builtin_fma(-kT1, a.y, -a.x), __builtin_fma(kT1, a.x, -a.y));
}
// dft4(a0, a1, a2, a3) for a1 = kC1 p1, a2 = kR2 u2, a3 = kC1 p3
__device__ __forceinline__ void dft4_r2c(double2 &a0, double2 p1, double2 u2, double2 &a2, double2 p3,
                                         double2 &o1, double2 &o3) {
    double2 t0, t1;
    fma_pm(a0, u2, t0, t1);
    const double2 s = cadd(p1, p3), d = csub(p1, p3);
    a0 = make_double2(__builtin_fma(kC1, s.x, t0.x), __builtin_fma(kC1, s.y, t0.y));
    a2 = make_double2(__builtin_fma(-kC1, s.x, t0.x), __builtin_fma(-kC1, s.y, t0.y));
    // t3 = -i kC1 d
    o1 = make_double2(__builtin_fma(kC1, d.y, t1.x), __builtin_fma(-kC1, d.x, t1.y));
    o3 = make_double2(__builtin_fma(-kC1, d.y, t1.x), __builtin_fma(kC1, d.x, t1.y));
}

// forward 16-point DFT, natural order in and out (4 x 4 Cooley-Tukey)
__device__ __forceinline__ void dft16(double2 (&a)[16]) {
    // radix-4 over n1 for each n2: slot 4*n1 + n2 -> slot 4*k1 + n2
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(a[n2], a[4 + n2], a[8 + n2], a[12 + n2]);
    // twiddles W16^(n2*k1), slot 4*k1 + n2, then radix-4 over n2 for each k1:
    // slot 4*k1 + k2 holds X[k1 + 4*k2].  The W16^2 = W8^1 and W16^6 = W8^3
    // rotations keep their sqrt(1/2) pending into the radix-4 (dft4_r13 and
    // the inline forms for rows 1 and 3).
    a[5] = w16<1>(a[5]);
    a[7] = w16<3>(a[7]);
    a[10] = w16<4>(a[10]);
    a[13] = w16<3>(a[13]);
    a[15] = w16<9>(a[15]);
    dft4(a[0], a[1], a[2], a[3]);
    dft4_r2(a[4], a[5], rot8_1(a[6]), a[6], a[7]); // row 1: (a4, a5 w1, kR2 rot8_1(a6), a7 w3)
    {
        // row 2: (a8, kR2 rot8_1(a9), -i a10, kR2 rot8_3(a11))
        double2 o1, o3;
        dft4_r13(a[8], rot8_1(a[9]), a[10], rot8_3(a[11]), o1, o3);
        a[9] = o1;
        a[11] = o3;
    }
    dft4_r2(a[12], a[13], rot8_3(a[14]), a[14], a[15]); // row 3: (a12, a13 w3, kR2 rot8_3(a14), a15 w9)
    double2 t[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) t[k1 + 4 * k2] = a[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = t[i];
}


// forward 8-point DFT, natural order in and out (radix-2 x 4)
__device__ __forceinline__ void dft8(double2 (&a)[8]) {
    double2 b[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b[k] = cadd(a[k], a[k + 4]);
        b[k + 4] = csub(a[k], a[k + 4]);
    }
    b[6] = mul_mi(b[6]); // W8^2
    dft4(b[0], b[1], b[2], b[3]);
    // (b4, b5 W8^1, b6, b7 W8^3) with the sqrt(1/2) of W8^1 and W8^3 folded into FMAs
    dft4_r13(b[4], rot8_1(b[5]), b[6], rot8_3(b[7]), b[5], b[7]);
    a[0] = b[0];
    a[2] = b[1];
    a[4] = b[2];
    a[6] = b[3];
    a[1] = b[4];
    a[3] = b[5];
    a[5] = b[6];
    a[7] = b[7];
}

// a[r] *= w1^r, r = 1..15, powers by an odd/even chain (w^(2i+1) = w^(2i-1) w^2):
// 4 live values, <= 8 products deep (error ~1e-15)
__device__ __forceinline__ void twiddle16(double2 (&a)[16], double2 w1) {
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

// w[r] = w1^r, r = 1..15, by twiddle16's chain (the same values, bit for bit)
__device__ __forceinline__ void powers16(double2 w1, double2 (&w)[16]) {
    const double2 w2 = cmul(w1, w1);
    w[1] = w1;
    w[2] = w2;
#pragma unroll
    for (int r = 3; r < 15; r += 2) {
        w[r] = cmul(w[r - 2], w2);
        w[r + 1] = cmul(w[r - 1], w2);
    }
    w[15] = cmul(w[13], w2);
}

__device__ __forceinline__ void apply16(double2 (&a)[16], const double2 (&w)[16]) {
#pragma unroll
    for (int r = 1; r < 16; ++r) a[r] = cmul(a[r], w[r]);
}

// w[r] = w1^r, r = 1..7 (depth <= 3)
__device__ __forceinline__ void powers8(double2 w1, double2 (&w)[8]) {
    w[1] = w1;
    w[2] = cmul(w1, w1);
    w[3] = cmul(w[2], w1);
    w[4] = cmul(w[2], w[2]);
    w[5] = cmul(w[4], w1);
    w[6] = cmul(w[4], w[2]);
    w[7] = cmul(w[4], w[3]);
}

__device__ __forceinline__ void twiddle8(double2 (&a)[8], const double2 (&w)[8]) {
#pragma unroll
    for (int r = 1; r < 8; ++r) a[r] = cmul(a[r], w[r]);
}

// The wave-local exchanges: LDS operations of one wave execute in order, so
// only the compiler must be kept from moving them across (rocPRIM's
// wave_barrier idiom).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS layouts inside one column block of 512 (index in 16-B units); XOR
// swizzles keep every exchange bank-conflict free (scripts/fft_lds_sim.py)
__device__ __forceinline__ int fx1(int l, int d1) { return 64 * d1 + (l ^ (8 * d1)); }
__device__ __forceinline__ int fx2(int l1, int d1, int e1) {
    return 64 * e1 + 8 * d1 + (l1 ^ (((d1 >> 1) & 1) | ((e1 & 3) << 1)));
}
__device__ __forceinline__ int fx3(int d1, int e1, int b0) { return 64 * e1 + 8 * b0 + d1; }
__device__ __forceinline__ int fx4(int d1, int b0, int g0) {
    return 64 * g0 + 8 * b0 + (d1 ^ (((b0 >> 1) & 1) | ((g0 & 3) << 1)));
}

// Samples of one unit: v[r] = (x_seg[2m], x_seg[2m+1]), m = j + 512 r, x_seg[i] =
// x[n0 - half + i].  Raw buffer loads through a range-checked resource over the
// loaded window [x_lo, x_hi): offsets outside it -- including "negative" ones,
// which wrap to huge unsigned offsets -- read 0.  That is the zero padding of
// FilterCore.h's shortened edge sums, with no branches.
// NR float2 per thread: 16 for L = 16 384, 32 for fir_fft32.hpp's L = 32 768.
template <int NR>
__device__ __forceinline__ void fft_load_unit(const DirectParams &p, int ch, int64_t n0, int j,
                                              float2 (&v)[NR]) {
    constexpr int kSeg = 1024 * NR; // real samples per segment
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(x), (short)0, (int)((p.x_hi - p.x_lo) * 4), 0x00020000);
    const int64_t w0 = n0 - p.half - p.x_lo; // window start inside the loaded range
    const int off0 = (int)(w0 * 4) + 8 * j;   // may be negative
    if (w0 >= 0 && w0 + kSeg <= p.x_hi - p.x_lo) {
        // interior unit (all but the first and last of a range): cached
        // dwordx2 loads (4-byte aligned is enough for buffer loads)
#pragma unroll
        for (int r = 0; r < NR; ++r)
            v[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off0 + 8 * 512 * r, 0, 0));
    } else {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int off = off0 + 8 * 512 * r;
            // aux bit 31 = volatile: keeps the two dword loads from being merged
            // into one dwordx2, whose range check is all-or-nothing (a pair
            // straddling the window start would lose its in-range sample)
            v[r].x = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, (int)0x80000000));
            v[r].y = __int_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, (int)0x80000000));
        }
    }
}

// W_L^(k_i) = W_L^(k_0) W_16^i for the pair in slot i (k_i = k_0 + 1024 i)
__device__ __forceinline__ double2 fft_pair_w(double2 wbase, int i) {
    switch (i) {
    case 1: return cmul(wbase, make_double2(kC1, -kS1));
    case 2: return w16<2>(wbase);
    case 3: return cmul(wbase, make_double2(kS1, -kC1));
    case 4: return mul_mi(wbase);
    case 5: return cmul(wbase, make_double2(-kS1, -kC1));
    case 6: return w16<6>(wbase);
    case 7: return cmul(wbase, make_double2(-kC1, -kS1));
    default: return wbase;
    }
}

// One bin pair of the real split + filter multiply + merge (conj trick
// applied): P = Z_k, Q = Z_{M-k}; S2 = 2S, D2 = 2D from the pair table.
__device__ __forceinline__ void fft_pair(double2 P, double2 Q, double2 W, double2 S2, double2 D2,
                                         double2 &oP, double2 &oQ) {
    const double2 P1 = make_double2(__builtin_fma(D2.x, W.y, S2.x), __builtin_fma(D2.y, W.y, S2.y));
    const double2 Q2 = make_double2(__builtin_fma(-D2.x, W.y, S2.x), __builtin_fma(-D2.y, W.y, S2.y));
    const double2 P2 = make_double2(-D2.y * W.x, D2.x * W.x);
    const double2 Zm = cconj(Q);
    oP = cconj(cadd(cmul(P, P1), cmul(Zm, P2)));
    oQ = csub(cmul(Zm, Q2), cmul(P, P2));
}

// The same pair for a linear-phase (symmetric) filter in zero-phase form
// (kFftOutSym): G is real, so 2S = s2 and 2D = d2 are real, P1 = p1 and Q2 =
// q2 real and P2 = i p2 imaginary, p1 = s2 + d2 Im W, q2 = s2 - d2 Im W, p2 =
// d2 Re W.  The table holds p1, q2, p2 per bin (kFftSymPQ, kFftSymP2): 8 f64
// operations per pair instead of ~26.
__device__ __forceinline__ void fft_pair_sym(double2 P, double2 Q, double p1, double q2, double p2,
                                             double2 &oP, double2 &oQ) {
    // oP = conj(P p1 + conj(Q) i p2),  oQ = conj(Q) q2 - P i p2
    oP = make_double2(__builtin_fma(p1, P.x, p2 * Q.y), -__builtin_fma(p1, P.y, p2 * Q.x));
    oQ = make_double2(__builtin_fma(q2, Q.x, p2 * P.y), -__builtin_fma(q2, Q.y, p2 * P.x));
}

// Wave 0's special lane (kFftSpecialLane) holds the self-paired tasks: A =
// column-0 task (d1, e1) = (0, 4), bins 512 + 1024 e2, pairs (A_i, A_7-i); B =
// task (0, 0), bins 1024 e2, pairs (B_i, B_8-i) with B_0 and B_4 self-paired.
// Its registers are permuted (per-lane selects) into the generic layout
// (P = x0[i], Q = x1[7-i]) so every lane runs the same pair loop:
//   x0 = [A0 A1 A2 A3 B0 B1 B2 B3],  x1 = [B5 B6 B7 B0 A4 A5 A6 A7]
// slots 0..3: k = 512 + 1024 i (W base W_L^512); slots 4..7: k = 1024 (i-4)
// (W base +i = W_16^-4); B_4 (k = M/2) is done apart.  Each chain reads every
// register before overwriting it, so no temporaries are needed.
__device__ __forceinline__ void fft_w0_permute_in(double2 (&x0)[8], double2 (&x1)[8], bool sp) {
    x1[4] = csel(sp, x0[4], x1[4]); // (B4 was taken out by the caller)
    x0[4] = csel(sp, x1[0], x0[4]);
    x1[0] = csel(sp, x1[5], x1[0]);
    x1[5] = csel(sp, x0[5], x1[5]);
    x0[5] = csel(sp, x1[1], x0[5]);
    x1[1] = csel(sp, x1[6], x1[1]);
    x1[6] = csel(sp, x0[6], x1[6]);
    x0[6] = csel(sp, x1[2], x0[6]);
    x1[2] = csel(sp, x1[7], x1[2]);
    x1[7] = csel(sp, x0[7], x1[7]);
    x0[7] = csel(sp, x1[3], x0[7]);
    x1[3] = csel(sp, x0[4], x1[3]);
}
// Inverse of the above on the pair outputs (x1[3] holds a duplicate of B0's
// output and is dropped); v4 = the output for B_4.
__device__ __forceinline__ void fft_w0_permute_out(double2 (&x0)[8], double2 (&x1)[8], bool sp, double2 v4) {
    x1[3] = csel(sp, x0[7], x1[3]);
    x0[7] = csel(sp, x1[7], x0[7]);
    x1[7] = csel(sp, x1[2], x1[7]);
    x1[2] = csel(sp, x0[6], x1[2]);
    x0[6] = csel(sp, x1[6], x0[6]);
    x1[6] = csel(sp, x1[1], x1[6]);
    x1[1] = csel(sp, x0[5], x1[1]);
    x0[5] = csel(sp, x1[5], x0[5]);
    x1[5] = csel(sp, x1[0], x1[5]);
    x1[0] = csel(sp, x0[4], x1[0]);
    x0[4] = csel(sp, x1[4], x0[4]);
    x1[4] = csel(sp, v4, x1[4]);
}

// The fused peak leaves a workgroup as ONE atomic per channel: each wave puts
// the max of its running per-lane peak into its LDS slot (fft_peak_stage),
// and after the next workgroup barrier thread 0 folds the 8 slots into one
// atomicMax (fft_peak_commit).  One atomic per wave -- 2 048 same-address
// atomics when every workgroup crosses into the next channel in the same
// round -- stalled that round by ~25 % (tools/launch_trace.hip).
__device__ __forceinline__ void fft_peak_stage(float *pk_lds, float pk) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) pk = fmaxf(pk, __shfl_xor(pk, s, 64));
    if ((threadIdx.x & 63) == 0) pk_lds[threadIdx.x >> 6] = pk;
}
// thread 0 only, after a barrier that follows every wave's fft_peak_stage
__device__ __forceinline__ void fft_peak_commit(const DirectParams &p, int ch, const float *pk_lds) {
    float pk = pk_lds[0];
#pragma unroll
    for (int w = 1; w < kFftNT / 64; ++w) pk = fmaxf(pk, pk_lds[w]);
    atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(pk));
}

// A previous file's normalize (ProcessFile.cp:98-101), carried by this
// launch: its outputs y[0, count) (contiguous, 16-B aligned) are rescaled by
// 1/peak iff max(peak[0, npeak)) > 1 or force -- normalize_kernel's rule and
// arithmetic, (float)((double)v * (1.0 / peak)), so bit-identical.  Unit u
// takes y[u slice, (u + 1) slice); the older waves of the workgroup (0..3)
// do it while they wait at the segment's second barrier for the younger
// ones (CHANGELOG.md s8 timeline), so a batch step needs one normalize pass
// (its last file's) instead of one per file.
struct FftNrm {
    float *y = nullptr;
    const unsigned *peak = nullptr;
    int64_t count = 0;
    int64_t slice = 0; // floats per unit, a multiple of 1024 (fft_launch)
    int32_t npeak = 0;
    int32_t force = 0;
};
// The older waves load, rescale and store their unit's slice while they wait
// at the segment's second barrier; the stores' completion is waited for only
// at the next unit's output stores.  Branch-free: a buffer resource over
// exactly the slice drops the lanes past its end (a divergent guard made the
// compiler wait for every earlier load before each one).  kNrmK 16-byte
// loads per thread, all in flight: slices of up to 14 336 floats
// (fft_nrm_fusable).  Non-temporal: the 8 B/sample stream must not evict the
// pair table and the halo samples the filter re-reads from L2.  (Deferring
// the rescale to the next barrier 1 kept kNrmK float4 live across the final
// phase: 256 VGPRs and scratch spills.)
constexpr int kNrmK = 14;
// fir_fft32r_kernel's halves: up to kNrmK32 blocks of 1 024 floats each, so a
// 60-min stereo file (15 blocks per half at 4 001 taps) still fuses
constexpr int kNrmK32 = 16;
constexpr int kNrmLoadAux = kNtStore; // the slice's loads: nt, as its stores
constexpr int kVmcntNrm = 0x0F70 | kNrmK; // s_waitcnt vmcnt(kNrmK): the slice's stores may stay in flight
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fft_nrm_rsrc(const FftNrm &nrm, int u, bool active = true) {
    const int64_t s0 = (int64_t)u * nrm.slice;
    const int64_t s1 = s0 + nrm.slice < nrm.count ? s0 + nrm.slice : nrm.count;
    const int len = active && s1 > s0 ? (int)(s1 - s0) : 0;
    return __builtin_amdgcn_make_buffer_rsrc(nrm.y + (s0 < nrm.count ? s0 : 0), (short)0, 4 * (len & ~3), 0x00020000);
}
// unconditional for every wave (an inactive one loads through an empty
// resource: no memory traffic), so v is defined on every path and never
// live across the column phase
template <int K = kNrmK>
__device__ __forceinline__ void fft_nrm_load(const FftNrm &nrm, int u, int t, bool active, float4 (&v)[K]) {
    const __amdgpu_buffer_rsrc_t r = fft_nrm_rsrc(nrm, u, active);
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, 16 * t + 4096 * k, 0, kNrmLoadAux));
}
template <int K = kNrmK>
__device__ __forceinline__ void fft_nrm_store(const FftNrm &nrm, int u, int t, double gain, float4 (&v)[K]) {
    const __amdgpu_buffer_rsrc_t r = fft_nrm_rsrc(nrm, u);
    using b128_t = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v[k].x = (float)((double)v[k].x * gain);
        v[k].y = (float)((double)v[k].y * gain);
        v[k].z = (float)((double)v[k].z * gain);
        v[k].w = (float)((double)v[k].w * gain);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128_t, v[k]), r, 16 * t + 4096 * k, 0, kNtStore);
    }
    // the last 1..3 floats when count is not a multiple of 4
    const int64_t s0 = (int64_t)u * nrm.slice;
    const int64_t s1 = s0 + nrm.slice < nrm.count ? s0 + nrm.slice : nrm.count;
    const int64_t tail = nrm.count & ~(int64_t)3;
    if (s1 == nrm.count && tail >= s0 && tail + t < nrm.count)
        nrm.y[tail + t] = (float)((double)nrm.y[tail + t] * gain);
}

// Column phase of one 8192-point transform held in the LDS work array
// (DESIGN.md s4.2): wave w owns the two columns in LDS slots 2w and 2w + 1 and
// runs their 512-point DFTs as 8 x 8 x 8 with wave-local exchanges (stages A,
// B), stage C per task, the pair step in registers, then the inverse stages
// A', B', C' back into the same slots.  LDS in, LDS out: the workgroup
// barriers around it are the caller's.  tk_all: this thread's task word;
// pair: the pair table of this transform; c8: the special lane's bin-M/2
// coefficient.  odd (wave-uniform): the transform has no self-paired bins
// (fir_fft32.hpp half O: columns w and 15 - w in every wave, task B the
// mirror of task A), so wave 0 runs the generic pair loop.  after_pair() runs
// between the pair step and stage A' (the caller's prefetch, or nothing).
// kReuseTw: the zero-phase form keeps stage A's and B's twiddle powers for A'
// and B' (56 VGPRs across the pair step; off where the caller parks data).
template <int kOut, bool kReuseTw = true, class AfterPair>
__device__ __forceinline__ void fft_columns(double2 *flds, const double2 *twl, const double2 *__restrict__ pair,
                                            uint32_t tk_all, double2 c8, bool odd, int j, int rnd,
                                            AfterPair &&after_pair) {
    (void)rnd; // phase stamps only (LCFIR_FFT_TRACE)
    const int lane = j & 63;
    const int w = j >> 6;
    // the wave's two columns in adjacent slots
    double2 *blk0 = flds + 512 * (2 * w);
    double2 *blk1 = blk0 + 512;
    double2 x0[8], x1[8]; // the wave's two columns (later: tasks A and B)
    double2 tws[8];
    // Stages A and B run as a two-column software pipeline: a column's
    // exchange reads are issued right behind its writes, and the other
    // column's arithmetic covers their latency (counted lgkmcnt waits).
    // ---- stage A: lane l holds b = l + 64 t; radix-8 over t -> d1; * W_512^(l d1)
    const int l1 = lane & 7, d1s = lane >> 3; // the stage-B lane (l1, d1)
#pragma unroll
    for (int t = 0; t < 8; ++t) x0[t] = blk0[lane + 64 * t];
#pragma unroll
    for (int t = 0; t < 8; ++t) x1[t] = blk1[lane + 64 * t];
    powers8(twl[512 + lane], tws);
    double2 tws_a[8]; // W_512^(lane r): stage A' of task A needs the same powers (waves 1..7, wave 0 lanes < 32)
    if constexpr (kOut == kFftOutSym && kReuseTw) {
#pragma unroll
        for (int r = 1; r < 8; ++r) tws_a[r] = tws[r];
    }
    dft8(x0);
    twiddle8(x0, tws);
#pragma unroll
    for (int d1 = 0; d1 < 8; ++d1) blk0[fx1(lane, d1)] = x0[d1];
    wave_lds_sync();
#pragma unroll
    for (int l2 = 0; l2 < 8; ++l2) x0[l2] = blk0[fx1(l1 + 8 * l2, d1s)];
    __builtin_amdgcn_sched_barrier(0);
    dft8(x1);
    twiddle8(x1, tws);
#pragma unroll
    for (int d1 = 0; d1 < 8; ++d1) blk1[fx1(lane, d1)] = x1[d1];
    wave_lds_sync();
#pragma unroll
    for (int l2 = 0; l2 < 8; ++l2) x1[l2] = blk1[fx1(l1 + 8 * l2, d1s)];
    __builtin_amdgcn_sched_barrier(0);
    FFT_STAMP(5);
    // ---- stage B: lane (l1, d1) has gathered l2; radix-8 -> e1; * W_64^(l1 e1)
    powers8(twl[512 + 8 * l1], tws);
    double2 tws_b[8]; // W_64^(l1 r): stage B' (d1 = lane & 7 = l1) needs the same powers
    if constexpr (kOut == kFftOutSym && kReuseTw) {
#pragma unroll
        for (int r = 1; r < 8; ++r) tws_b[r] = tws[r];
    }
    dft8(x0);
    twiddle8(x0, tws);
#pragma unroll
    for (int e1 = 0; e1 < 8; ++e1) blk0[fx2(l1, d1s, e1)] = x0[e1];
    __builtin_amdgcn_sched_barrier(0);
    dft8(x1);
    twiddle8(x1, tws);
#pragma unroll
    for (int e1 = 0; e1 < 8; ++e1) blk1[fx2(l1, d1s, e1)] = x1[e1];
    wave_lds_sync();
    FFT_STAMP(6);
    // ---- pair-table loads, issued ahead of stage C (L2 latency off the path)
    constexpr bool kSym = kOut == kFftOutSym;
    double2 qs[kSym ? 1 : 8], qd[kSym ? 1 : 8]; // 2 S and 2 D of the pair in slot i
    double2 qpq[kSym ? 8 : 1], qp2[kSym ? 4 : 1]; // kSym: (p1, q2) of slot i, p2 of slots 2m, 2m+1
    double2 wbase;                                // W_L^k of slot 0 (general form)
    if constexpr (kSym) {
        const double2 *t = pair + j;
#pragma unroll
        for (int i = 0; i < 8; ++i) qpq[i] = t[kFftSymPQ + 512 * i]; // one 16-byte load per slot
#pragma unroll
        for (int m = 0; m < 4; ++m) qp2[m] = t[kFftSymP2 + 512 * m];
    } else {
        const double2 *t = pair + j;
        wbase = pair[2 * kFftPairSlots * 512 + j];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            qs[i] = t[512 * i];
            qd[i] = t[kFftPairSlots * 512 + 512 * i];
        }
    }
    __builtin_amdgcn_sched_barrier(0); // keep the loads ahead of stage C
    // ---- stage C: per task, radix-8 over l1 -> e2: x0[e2] = X[kA], x1[e2] = X[kB]
    const uint32_t tk = tk_all;
    const int cA = tk & 15, dA = (tk >> 4) & 7, eA = (tk >> 7) & 7; // cA, cB: LDS slots
    const int cB = (tk >> 10) & 15, dB = (tk >> 14) & 7, eB = (tk >> 17) & 7;
    {
        const double2 *ba = flds + 512 * cA, *bb = flds + 512 * cB;
#pragma unroll
        for (int l1 = 0; l1 < 8; ++l1) x0[l1] = ba[fx2(l1, dA, eA)];
#pragma unroll
        for (int l1 = 0; l1 < 8; ++l1) x1[l1] = bb[fx2(l1, dB, eB)];
    }
    dft8(x0);
    dft8(x1);
    FFT_STAMP(7);
    // ---- pair step in registers: pairs (x0[i], x1[7-i]); outputs conj(V).
    // The real split, the multiply by G and the merge collapse to
    //   conj(V_k) = conj(Z_k P1 + conj(Z_{M-k}) P2),  conj(V_{M-k}) = conj(Z_{M-k}) Q2 - Z_k P2
    // with S = G_k + conj(G_{M-k}), D = G_k - conj(G_{M-k}), W = W_L^k:
    //   P1 = 2 (S + D Im W),  P2 = 2i D Re W,  Q2 = 2 (S - D Im W)
    // General form: the table holds 2S and 2D per (slot, thread) (host, long
    // double) and W comes from one per-thread base times W_16^i.  Zero-phase
    // form: the table holds P1 = p1, Q2 = q2 and P2 / i = p2 per bin.
    {
        // Wave 0 (a scalar, wave-uniform branch) permutes its special lane
        // into the generic layout first (fft_w0_permute_in).
        const bool w0 = !odd && __builtin_amdgcn_readfirstlane(w) == 0;
        const bool sp = w0 && lane == kFftSpecialLane;
        double2 wb_hi = wbase; // W base of slots 4..7 (general form; the zero-phase table has per-bin p1, q2, p2)
        double2 v4 = x1[4];    // special lane: B_4, bin M/2 (slot 8, W = -i): P1 = 2S - 2D, P2 = 0
        if (w0) {
            v4 = cconj(cmul(v4, c8)); // a kernel argument (SGPRs: no L2 wait here)
            if constexpr (!kSym) wb_hi = csel(sp, make_double2(0.0, 1.0), wbase);
            fft_w0_permute_in(x0, x1, sp);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (kSym)
                fft_pair_sym(x0[i], x1[7 - i], qpq[i].x, qpq[i].y, (i & 1) ? qp2[i >> 1].y : qp2[i >> 1].x, x0[i],
                             x1[7 - i]);
            else
                fft_pair(x0[i], x1[7 - i], fft_pair_w(i < 4 ? wbase : wb_hi, i), qs[i], qd[i], x0[i],
                         x1[7 - i]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (w0) fft_w0_permute_out(x0, x1, sp, v4);
    }

    FFT_STAMP(8);
    after_pair(); // the caller's prefetch of the next unit's samples

    // ---- inverse stage A': per task radix-8 over e2 -> beta0; * W_512^(beta0 d')
    {
        double2 *ba = flds + 512 * cA, *bb = flds + 512 * cB;
        if constexpr (kOut == kFftOutSym && kReuseTw) {
            // task A's d' = dA + 8 eA is the lane except in wave 0's column-0
            // lanes (kFftWave0C0) of an even transform: a wave-uniform choice
            if (odd || __builtin_amdgcn_readfirstlane(w) != 0) {
#pragma unroll
                for (int r = 1; r < 8; ++r) tws[r] = tws_a[r];
            } else {
                powers8(twl[512 + dA + 8 * eA], tws);
            }
        } else {
            powers8(twl[512 + dA + 8 * eA], tws);
        }
        dft8(x0);
        twiddle8(x0, tws);
#pragma unroll
        for (int b0 = 0; b0 < 8; ++b0) ba[fx3(dA, eA, b0)] = x0[b0];
        __builtin_amdgcn_sched_barrier(0);
        powers8(twl[512 + dB + 8 * eB], tws);
        dft8(x1);
        twiddle8(x1, tws);
#pragma unroll
        for (int b0 = 0; b0 < 8; ++b0) bb[fx3(dB, eB, b0)] = x1[b0];
    }
    wave_lds_sync();
    FFT_STAMP(9);
    // ---- stage B': lane (d1, beta0) gathers e1; radix-8 -> gamma0; * W_64^(gamma0 d1)
    // (wave 0's column-0 block was written by both tasks: both writes precede
    // these reads).  B' and C' are software-pipelined like A and B.
    {
        const int d1 = lane & 7, b0 = lane >> 3;  // stage-B' lane
        const int rb0 = lane & 7, rg0 = lane >> 3; // stage-C' lane rho = beta0 + 8 gamma0
#pragma unroll
        for (int e1 = 0; e1 < 8; ++e1) x0[e1] = blk0[fx3(d1, e1, b0)];
#pragma unroll
        for (int e1 = 0; e1 < 8; ++e1) x1[e1] = blk1[fx3(d1, e1, b0)];
        if constexpr (kOut == kFftOutSym && kReuseTw) {
#pragma unroll
            for (int r = 1; r < 8; ++r) tws[r] = tws_b[r]; // registers to spare in this form
        } else {
            powers8(twl[512 + 8 * d1], tws);
        }
        dft8(x0);
        twiddle8(x0, tws);
#pragma unroll
        for (int g0 = 0; g0 < 8; ++g0) blk0[fx4(d1, b0, g0)] = x0[g0];
        wave_lds_sync();
#pragma unroll
        for (int dd = 0; dd < 8; ++dd) x0[dd] = blk0[fx4(dd, rb0, rg0)];
        __builtin_amdgcn_sched_barrier(0);
        dft8(x1);
        twiddle8(x1, tws);
#pragma unroll
        for (int g0 = 0; g0 < 8; ++g0) blk1[fx4(d1, b0, g0)] = x1[g0];
        wave_lds_sync();
#pragma unroll
        for (int dd = 0; dd < 8; ++dd) x1[dd] = blk1[fx4(dd, rb0, rg0)];
        __builtin_amdgcn_sched_barrier(0);
    }
    FFT_STAMP(10);
    // ---- stage C': lane rho = beta0 + 8 gamma0 has gathered d1; radix-8 -> gamma1
    dft8(x0);
#pragma unroll
    for (int g1 = 0; g1 < 8; ++g1) blk0[lane + 64 * g1] = x0[g1]; // b = lane + 64 gamma1
    __builtin_amdgcn_sched_barrier(0);
    dft8(x1);
#pragma unroll
    for (int g1 = 0; g1 < 8; ++g1) blk1[lane + 64 * g1] = x1[g1];
    FFT_STAMP(11);
}

// Persistent: one workgroup per CU walks the units u = blockIdx.x + i * gridDim.x
// of the nch x nseg (channel, segment) grid.  The next unit's samples are
// loaded during the current unit's final phase, so HBM latency is off the path.
//
// Inside a wave the two columns are software-pipelined through every
// wave-local exchange: column 0's LDS writes are issued before column 1's
// arithmetic, which then runs while the LDS drains them (sched_barrier pins
// the order; the LDS executes one wave's operations in issue order, so each
// read still follows the writes it needs).
//
// kOut selects what a unit does with its outputs (filters longer than one
// partition run one launch per partition over the same range, fft_launch):
//   kFftOutF32   : RNE to f32 into y, fused peak (single-partition filters);
//   kFftOutFirst : write the f64 partial sum into the scratch p.y64;
//   kFftOutAdd   : add it to p.y64;
//   kFftOutLast  : RNE(p.y64 + partial) to f32 into y, fused peak.
// c8 = the special lane's bin-M/2 coefficient 2S - 2D of this pair table.
// kNrm: the launch also rescales a previous file's outputs (FftNrm).
template <int kOut, bool kNrm = false>
__global__ __launch_bounds__(kFftNT) void fir_fft_f64_kernel(DirectParams p, const double2 *__restrict__ pair,
                                                            const double2 *__restrict__ tw,
                                                            const uint32_t *__restrict__ task, int B,
                                                            FftGrid gd, double2 c8, FftNrm nrm) {
    extern __shared__ double2 flds[];
    FFT_USTAMP(0);
    // kNrm: the normalize decision, once per launch (uniform)
    bool nrm_on = false;
    double nrm_gain = 1.0;
    if constexpr (kNrm) {
        float pkv = 0.0f;
        for (int i = 0; i < nrm.npeak; ++i) pkv = fmaxf(pkv, __uint_as_float(nrm.peak[i]));
        nrm_on = (pkv > 1.0f || nrm.force) && pkv > 0.0f;
        nrm_gain = 1.0 / (double)pkv;
        __builtin_amdgcn_s_setprio(1); // the older waves drop to 0 for their normalize slices
    }

    double2 *twl = flds + kFftM; // the kFftTw twiddles, LDS-resident
    for (int i = threadIdx.x; i < kFftTw; i += kFftNT) twl[i] = tw[i];
    float2 v[16]; // samples of the unit about to start
    {
        const int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units); // < units: the grid is <= units
        const int c = fft_div(u, gd);
        fft_load_unit(p, c, p.seg0 + (int64_t)(u - c * gd.nseg) * B, threadIdx.x, v);
    }
    // vmcnt counts loads and stores together, in issue order, and the wait
    // pass merges the loop's entry and back edge path-insensitively.  Both
    // paths therefore reach the loop head with every prefetch load retired
    // (here, and just before each unit's output stores), so stage 1 never
    // waits on the previous unit's stores.
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    // task word of this thread (exchange-2 tasks; fixed for the whole launch)
    uint32_t tk_all = task[threadIdx.x];
    asm volatile("" : "+v"(tk_all));
    float pk_run = 0.0f; // running max |y| of channel pk_ch over this lane's outputs
    int pk_ch = -1;
    float *pk_lds = reinterpret_cast<float *>(twl + kFftTw); // per-wave peaks (fft_peak_stage)
    int pk_pending = -1; // channel whose staged per-wave peaks await thread 0's commit
    double2 wt[16]; // W_8192^(j c), c = 1..15: built in each final phase, used again by the next stage 1
    powers16(twl[threadIdx.x], wt);
    int rnd = 0; // round: this workgroup's unit ordinal
    for (int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units); u < gd.units;
         u = fft_unit32(++rnd, blockIdx.x, gridDim.x, gd.units)) {
    // Laundered thread index: everything derived from it is recomputed per
    // unit instead of being hoisted out of the loop (keeps pressure down).
    int j = threadIdx.x;
    asm volatile("" : "+v"(j));
    const int w = j >> 6; // the wave: its columns {w, 16 - w} (wave 0: {0, 8}), fft_columns
    const int ch = fft_div(u, gd);
    const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;
    FFT_STAMP(0);
    FFT_USTAMP(1 + rnd);

    // ---- stage 1: thread b = j, 16-point DFT over z[512 a + b] -> column c
    {
        double2 a[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = make_double2((double)v[r].x, (double)v[r].y);
        dft16(a);
        apply16(a, wt); // W_8192^(b c): the powers the previous unit's final phase built
        FFT_STAMP(1);
        // No barrier before this write: thread j overwrites exactly the
        // addresses flds[512 c + j] it read itself in the previous unit's
        // final phase, so program order already orders the two.
        FFT_STAMP(2);
#pragma unroll
        for (int c = 0; c < 16; ++c) flds[512 * fft_slot(c) + j] = a[c];
        FFT_STAMP(3);
        __syncthreads();
        // the previous channel's staged peaks (written before this barrier;
        // rewritten at the earliest after the next one)
        if (pk_pending >= 0) {
            if (threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
            pk_pending = -1;
        }
        FFT_STAMP(4);
    }

    fft_columns<kOut>(flds, twl, pair, tk_all, c8, false, j, rnd, [&] {
        // ---- prefetch the next unit's samples (consumed by its stage 1).
        // Unconditional (the last unit reloads itself): a conditional load
        // would keep the old v live across the whole loop body.
        const int un1 = fft_unit32(rnd + 1, blockIdx.x, gridDim.x, gd.units);
        const int un = un1 < gd.units ? un1 : u;
        const int cn = fft_div(un, gd);
        fft_load_unit(p, cn, p.seg0 + (int64_t)(un - cn * gd.nseg) * B, j, v);
    });
    if constexpr (kNrm) {
        // waves 0..3 reach this barrier well before waves 4..7: they spend
        // the wait on this unit's slice of the previous file's normalize
        // (loads, rescale and stores here; the stores' completion is waited
        // for only at the next unit's output stores, kVmcntNrm)
        if (nrm_on && w < 4) {
            // at priority 0 while the younger waves (1) finish their columns:
            // +1.8 % on config 5 (profiles/r02s3_fused_normalize_ab.txt)
            __builtin_amdgcn_s_setprio(0);
            float4 nv[kNrmK];
            fft_nrm_load(nrm, u, j, true, nv);
            fft_nrm_store(nrm, u, j, nrm_gain, nv);
            __builtin_amdgcn_s_setprio(1);
        }
        // an LDS-only barrier: __syncthreads() would first wait for those
        // global stores to complete (its release fence covers every space)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    } else {
        __syncthreads();
    }
    FFT_STAMP(12);

    // ---- final: thread b = j gathers its 16 columns, * W_8192^(b c), 16-point DFT -> v[512 a + b]
    double2 a[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) a[c] = flds[512 * fft_slot(c) + j];
    powers16(twl[j], wt); // kept for the next unit's stage 1 (same b = j)
    apply16(a, wt);
    dft16(a);
    FFT_STAMP(13);
    // ---- outputs: c[2m] = Re v'[m], c[2m+1] = -Im v'[m] (conj of the conj
    // trick), m = 512 r + j, valid for c >= T-1.  Range-checked buffer over
    // y[start, end): invalid lanes store to an out-of-range offset, which the
    // hardware drops (no branches).
    // the prefetch has landed long ago (see the loop head); kNrm: the older
    // waves leave their normalize slice's stores (the newest kNrmK) in flight
    if (kNrm && nrm_on && w < 4)
        __builtin_amdgcn_s_waitcnt(kVmcntNrm);
    else
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
        yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
    // valid outputs c in [cmin, cmax): [T-1, L) for the causal table, [half,
    // L - half) for the zero-phase one (kSym, fft_plan_build; an odd half
    // makes cmin odd)
    constexpr bool kSym = kOut == kFftOutSym;
    const int cmin = kSym ? p.half : p.ntaps - 1;
    const int cmax = kSym ? kFftL - p.half : kFftL;
    // (negative for outputs before `start`: the launch's segment grid starts
    // at p.seg0 <= start, fft_launch_group)
    const int64_t off = n0 - cmin - p.start; // offset (samples) of c[0] from start
    const int64_t oend = p.end - p.start;
    float pk = 0.0f;
    if constexpr (kOut == kFftOutF32 || kSym) {
    if (kSym && (cmin & 1) && n0 >= p.start && n0 + B <= p.end) {
        // the zero-phase form of an odd half: every output of this unit is
        // in [start, end), but the ends of [cmin, cmax) split a pair
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 2 * (j + 512 * r);
            const float f0 = (float)a[r].x, f1 = (float)(-a[r].y);
            const bool ok0 = c >= cmin && c < cmax, ok1 = c + 1 >= cmin && c + 1 < cmax;
            const int ob = (int)((off + c) * 4);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? ob : (int)0x80000000, 0, kNtStore);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ok1 ? ob + 4 : (int)0x80000000, 0,
                                                  kNtStore);
            pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
        }
    } else if (n0 >= p.start && n0 + B <= p.end) {
        // every output of this unit is in [start, end) and cmin, cmax are
        // even: the pair (c, c+1) is valid iff cmin <= c < cmax, so both
        // stores share one offset and may merge into a dwordx2.  (A resource
        // over the unit's B outputs, letting the range check drop the rest,
        // with a sign-bit mask for the peak removed the SGPR spills but
        // measured 2 % slower: the compares this form hoists fill VALU gaps
        // of the final DFT.)
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
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys,
                                                  ok0 ? (int)(o * 4) : (int)0x80000000, 0, kNtStore);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                  ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, kNtStore);
            pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
        }
    }
    } else {
        // partitioned filter: the f64 partial sums of outputs [start, end) live
        // in the scratch p.y64 (element 0 = output `start`, channel stride
        // y64_stride); every output belongs to exactly one unit per launch, so
        // the read-modify-write needs no atomics.  Invalid outputs use an
        // out-of-range offset: their loads return 0 and their stores drop.
        double *zb = p.y64 + (int64_t)ch * p.y64_stride;
        const __amdgpu_buffer_rsrc_t zs = __builtin_amdgcn_make_buffer_rsrc(
            zb, (short)0, (int)(oend * 8), 0x00020000);
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
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys,
                                                      ok0 ? (int)(o * 4) : (int)0x80000000, 0, kNtStore);
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
    // fused peak: a running per-lane max, staged (fft_peak_stage) only when
    // this workgroup moves to another channel and at the end -- a per-unit
    // atomic from every wave serialised on the peak slots and cost ~40 % of
    // the kernel.  Staging follows this unit's second barrier, so thread 0
    // has committed the previous staging (after the first) already.
    if (ch != pk_ch) {
        if (p.peak && pk_ch >= 0) {
            fft_peak_stage(pk_lds, pk_run);
            pk_pending = pk_ch;
            asm volatile("" : "+v"(pk_pending)); // a VGPR: SGPRs are the scarcer file here
        }
        pk_run = 0.0f;
        pk_ch = ch;
    }
    pk_run = fmaxf(pk_run, pk);
    FFT_STAMP(14);
    }
    FFT_USTAMP(1 + rnd);
    if (p.peak && pk_ch >= 0) {
        __syncthreads();
        if (pk_pending >= 0 && threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
        __syncthreads();
        fft_peak_stage(pk_lds, pk_run);
        __syncthreads();
        if (threadIdx.x == 0) fft_peak_commit(p, pk_ch, pk_lds);
    }
}

#include "fir_fft32.hpp"
#include "fir_fft32r.hpp"

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


// The host-side part of an FFT plan, from the taps alone (no device): the
// segment length, partitioning, pair tables, task words and twiddles the
// kernels read.  tests/cpp/fft_tables_dump.cpp writes them out for the CPU
// test that runs scripts/fft32_model.py's emulation of the kernel on them.
struct FftTables {
    int L = 0, halves = 1, parts = 1, tp = 0;
    bool sym = false, reg32 = false;
    std::vector<double2> pair; // parts x halves x kFftPairTable
    std::vector<uint32_t> task; // halves x 512
    std::vector<double2> c8;   // per partition
    std::vector<double2> tw;   // kFftTw or kFft32Tw
};

// fir_fft32r_kernel's tables (zero-phase, one partition, L = 32768): per
// thread t and pair slot i the zero-phase coefficients p1, q2, p2 of the bin in
// its R1 register i (the special lane: of its permuted x' list), the task
// words, and the twiddles W_16384^b, W_1024^b (b < 512), W_512^g (g < 16).
inline void r32_plan_tables(const std::vector<double> &taps, FftTables &T) {
    const int ntaps = (int)taps.size(), L = kFft32L, N = L / 2;
    const long double scale = 1.0L / (4.0L * (long double)N);
    const long double two_pi = 6.283185307179586476925286766559L;
    std::vector<long double> re((size_t)L, 0.0L), im((size_t)L, 0.0L);
    const int half = (ntaps - 1) / 2;
    for (int j = -half; j <= half; ++j)
        re[(size_t)((j + L) % L)] =
            ((long double)taps[(size_t)(half + j)] + (long double)taps[(size_t)(half - j)]) * 0.5L;
    detail::fft_ld(re, im);
    // p1, q2, p2 of bin k (fft_pair_sym; fft_plan_tables' zero-phase layout)
    auto coef = [&](int k, long double &p1, long double &q2, long double &p2, long double &c8v) {
        const long double gr = re[(size_t)k] * scale, hr = re[(size_t)(N - k)] * scale;
        const long double sr = gr + hr, dr = gr - hr;
        const long double a = -two_pi * (long double)k / (long double)L;
        p1 = 2 * sr + 2 * dr * sinl(a);
        q2 = 2 * sr - 2 * dr * sinl(a);
        p2 = 2 * dr * cosl(a);
        c8v = 2 * sr - 2 * dr;
    };
    T.pair.assign(kR32PairTable, make_double2(0.0, 0.0));
    T.task.resize(kFftNT);
    for (int t = 0; t < kFftNT; ++t) {
        T.task[(size_t)t] = r32_task_word(t);
        int bx[16], by[16];
        r32_task_bins(t, bx, by);
        if (t == kR32SpecialLane) {
            // x' = [R2 0..7, R1 1..7, R1 0] (fir_fft32r_kernel's permutation)
            int px[16];
            for (int i = 0; i < 8; ++i) px[i] = by[i];
            for (int i = 8; i < 15; ++i) px[i] = bx[i - 7];
            px[15] = bx[0];
            for (int i = 0; i < 16; ++i) bx[i] = px[i];
        }
        for (int i = 0; i < 16; ++i) {
            long double p1, q2, p2, c8v;
            coef(bx[i], p1, q2, p2, c8v);
            T.pair[(size_t)i * kFftNT + (size_t)t] = make_double2((double)p1, (double)q2);
            double *p2t = reinterpret_cast<double *>(&T.pair[(size_t)(16 + (i >> 1)) * kFftNT + (size_t)t]);
            p2t[i & 1] = (double)p2;
        }
    }
    {
        long double p1, q2, p2, c8v;
        coef(N / 2, p1, q2, p2, c8v);
        T.c8.assign(1, make_double2((double)c8v, 0.0));
    }
    T.tw.resize(kR32Tw);
    for (int b = 0; b < 512; ++b) {
        const long double a = -two_pi * (long double)b / 16384.0L, a16 = -two_pi * (long double)b / 1024.0L;
        T.tw[(size_t)(kR32TwB + b)] = make_double2((double)cosl(a), (double)sinl(a));
        T.tw[(size_t)(kR32TwB16 + b)] = make_double2((double)cosl(a16), (double)sinl(a16));
    }
    for (int g = 0; g < 16; ++g) {
        const long double a = -two_pi * (long double)g / 512.0L;
        T.tw[(size_t)(kR32TwG + g)] = make_double2((double)cosl(a), (double)sinl(a));
    }
    T.L = L;
    T.halves = 1;
    T.parts = 1;
    T.tp = ntaps;
    T.sym = true;
    T.reg32 = true;
}

inline FftTables fft_plan_tables(const std::vector<double> &taps, const FftTuning &tune) {
    const int ntaps = (int)taps.size();
    // segment length: the tuning's, else the filter's cheaper one per output;
    // L = 32768 runs fir_fft32.hpp's two 8192-point halves (bins of each parity)
    const int L = tune.seg_len ? tune.seg_len : fft_choose_seg_len(taps, tune);
    const int halves = L == kFft32L ? 2 : 1;
    const int Mf = L / 2; // complex transform length
    const int parts = fft_partition_count(ntaps, L);
    const int tp = parts == 1 ? ntaps : fft_partition_taps(ntaps, parts);
    const bool sym = fft_sym_eligible(taps, parts, tune);
    const long double scale = 1.0L / (4.0L * (long double)Mf);
    const long double two_pi = 6.283185307179586476925286766559L;
    // pair tables in consumption order: slot i of thread t holds bin k_i of
    // its task A (special lane: the permuted list; slot 8: k = M/2) as the
    // collapsed split/multiply/merge coefficients 2S, 2D, plus W_L^k in the
    // third field (the kernel reads slot 0's as its W base); the zero-phase
    // form stores fft_pair_sym's p1, q2, p2 per bin instead (kFftSymPQ, kFftSymP2).
    // Bin kappa of an 8192-point transform is k = kappa (L = 16384) or, half h
    // of L = 32768, k = 2 kappa + h; its partner is M - k in either case.
    FftTables T;
    std::vector<double2> &pair = T.pair, &c8 = T.c8;
    std::vector<uint32_t> &task = T.task;
    if (fft_reg32(L, parts, sym, tune)) {
        r32_plan_tables(taps, T);
        return T;
    }
    pair.resize((size_t)parts * halves * kFftPairTable);
    task.resize((size_t)halves * kFftNT);
    c8.resize((size_t)parts);
    auto cplx = [](long double r, long double i) { return make_double2((double)r, (double)i); };
    std::vector<long double> re((size_t)L), im((size_t)L);
    for (int part = 0; part < parts; ++part) {
        // G = FFT_L(g), g[j] = h_p[tp-1-j] with h_p[k] = h[part * tp + k] (0 past
        // the filter's end), zero padded; scaled by 1/(4M)
        std::fill(re.begin(), re.end(), 0.0L);
        std::fill(im.begin(), im.end(), 0.0L);
        if (!sym) {
            for (int i = 0; i < tp; ++i) {
                const int64_t k = (int64_t)part * tp + (tp - 1 - i);
                re[(size_t)i] = k < ntaps ? (long double)taps[(size_t)k] : 0.0L;
            }
        } else {
            // zero-phase form: g[j mod L] = h_sym[half + j], j in [-half, half],
            // h_sym = (h + reversed h) / 2 -- real and even, so G is real
            const int half = (ntaps - 1) / 2;
            for (int j = -half; j <= half; ++j)
                re[(size_t)((j + L) % L)] =
                    ((long double)taps[(size_t)(half + j)] + (long double)taps[(size_t)(half - j)]) * 0.5L;
        }
        detail::fft_ld(re, im);
        for (int h = 0; h < halves; ++h) {
            double2 *pt = pair.data() + ((size_t)part * halves + (size_t)h) * kFftPairTable;
            for (int t = 0; t < kFftNT; ++t) {
                const uint32_t tk = h == 0 ? fft_task_word(t) : fft32_task_word_odd(t);
                task[(size_t)h * kFftNT + (size_t)t] = tk;
                const int ca = h == 0 ? fft_slot_column(tk & 15) : fft32_slot_odd_column(tk & 15);
                const int da = (tk >> 4) & 7, ea = (tk >> 7) & 7;
                const bool sp = h == 0 && t == kFftSpecialLane;
                for (int i = 0; i < (h == 0 ? kFftPairSlots : 8); ++i) {
                    int kap;
                    if (i == 8) kap = kFftM / 2;
                    else if (!sp) kap = ca + 16 * (da + 8 * ea + 64 * i);
                    else kap = i < 4 ? 512 + 1024 * i : 1024 * (i - 4); // fft_w0_permute_in
                    const int k = halves == 1 ? kap : 2 * kap + h;
                    const long double gr = re[(size_t)k] * scale, gi = im[(size_t)k] * scale;
                    const long double hr = re[(size_t)(Mf - k)] * scale, hi = -im[(size_t)(Mf - k)] * scale;
                    const long double sr = gr + hr, si = gi + hi; // S = G_k + conj(G_{M-k})
                    const long double dr = gr - hr, di = gi - hi; // D = G_k - conj(G_{M-k})
                    const long double a = -two_pi * (long double)k / (long double)L;
                    const long double c = cosl(a), sn = sinl(a); // W = c + i sn
                    const size_t o = (size_t)i * kFftNT + (size_t)t;
                    if (!sym) {
                        pt[o] = cplx(2 * sr, 2 * si);
                        pt[(size_t)kFftPairSlots * kFftNT + o] = cplx(2 * dr, 2 * di);
                        pt[(size_t)2 * kFftPairSlots * kFftNT + o] = cplx(c, sn);
                    } else if (i < 8) {
                        // zero-phase layout: p1, q2, p2 per (slot, thread) (fft_pair_sym)
                        const long double p1 = 2 * sr + 2 * dr * sn, q2 = 2 * sr - 2 * dr * sn, p2 = 2 * dr * c;
                        pt[(size_t)kFftSymPQ + o] = cplx(p1, q2);
                        double *p2t =
                            reinterpret_cast<double *>(pt + kFftSymP2 + (size_t)(i >> 1) * kFftNT + (size_t)t);
                        p2t[i & 1] = (double)p2;
                    }
                    if (i == 8 && sp) c8[(size_t)part] = cplx(2 * sr - 2 * dr, sym ? 0.0L : 2 * si - 2 * di);
                }
            }
        }
    }
    // W_8192^i (i < 512), W_512^i (i < 64); L = 32768 adds W_16384^i (i < 512)
    std::vector<double2> &tw = T.tw;
    tw.resize((size_t)(halves == 2 ? kFft32Tw : kFftTw));
    for (int i = 0; i < 512; ++i) {
        const long double a = -two_pi * (long double)i / 8192.0L;
        tw[(size_t)i] = make_double2((double)cosl(a), (double)sinl(a));
    }
    for (int i = 0; i < 64; ++i) {
        const long double a = -two_pi * (long double)i / 512.0L;
        tw[(size_t)(512 + i)] = make_double2((double)cosl(a), (double)sinl(a));
    }
    if (halves == 2)
        for (int i = 0; i < 512; ++i) {
            const long double a = -two_pi * (long double)i / 16384.0L;
            tw[(size_t)(kFft32TwOdd + i)] = make_double2((double)cosl(a), (double)sinl(a));
        }
    T.L = L;
    T.halves = halves;
    T.parts = parts;
    T.tp = tp;
    T.sym = sym;
    return T;
}

inline bool fft_plan_build(FftPlan &plan, const double *d_taps, int ntaps, const FftTuning &tune, hipStream_t s,
                           std::string &err) {
    if (!fft_supported(ntaps)) {
        err = "tap count outside the FFT method's range";
        return false;
    }
    std::vector<double> taps((size_t)ntaps);
    if (hipMemcpyAsync(taps.data(), d_taps, sizeof(double) * (size_t)ntaps, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        err = "tap download failed";
        return false;
    }
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        cus > 0)
        plan.cus = cus;
    const FftTables T = fft_plan_tables(taps, tune);
    const std::vector<double2> &pair = T.pair, &tw = T.tw;
    const std::vector<uint32_t> &task = T.task;
    // stream-ordered on the ctx's own stream s (freed the same way, fft_plan_free)
    if (hipMallocAsync(reinterpret_cast<void **>(&plan.d_pair), sizeof(double2) * pair.size(), s) != hipSuccess ||
        hipMallocAsync(reinterpret_cast<void **>(&plan.d_tw), sizeof(double2) * tw.size(), s) != hipSuccess ||
        hipMallocAsync(reinterpret_cast<void **>(&plan.d_task), sizeof(uint32_t) * task.size(), s) != hipSuccess) {
        err = "hipMallocAsync for the FFT plan failed";
        return false;
    }
    if (hipMemcpyAsync(plan.d_pair, pair.data(), sizeof(double2) * pair.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipMemcpyAsync(plan.d_tw, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipMemcpyAsync(plan.d_task, task.data(), sizeof(uint32_t) * task.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        err = "FFT plan upload failed";
        return false;
    }
    plan.L = T.L;
    plan.ntaps = T.tp;
    plan.parts = T.parts;
    plan.sym = T.sym;
    plan.reg32 = T.reg32;
    plan.tune = tune;
    plan.B = T.L - T.tp + 1;
    plan.c8 = T.c8;
    plan.ready = true;
    return true;
}

// work array + twiddles + one f32 peak slot per wave (L = 32768: 145 KiB)
constexpr size_t fft_lds_bytes(int L = 16384) {
    return sizeof(double2) * (size_t)(kFftM + (L == kFft32L ? kFft32Tw : kFftTw)) + 4 * (kFftNT / 64);
}

// Outputs per launch.  The kernel addresses samples and outputs through raw
// buffer resources with 32-bit byte offsets (and 0x80000000 as its "drop this
// store" offset), so every launch's input window and output range must stay
// well under 2 GiB: longer ranges are split into chunks, each with its own
// narrowed input window.  Overlap-save is exact under any segmentation, and
// an output only needs x[out - half, out + half], inside its chunk's window.
// FftTuning::chunk lowers it (tests exercise the chunk seams with small values).
inline int64_t fft_chunk(const FftPlan &plan) {
    return plan.tune.chunk >= 4096 ? plan.tune.chunk : ((int64_t)1 << 28);
}

// work array + twiddles + 8 f32 peak slots + the special lane's 32 double2
constexpr size_t kR32LdsBytes = sizeof(double2) * (size_t)(kR32Work + kR32Tw + 2 + 32);

// Probe: fir_fft32r_kernel's phase hook (tools/fft32r_trace.hip passes its own)
template <int kOut, bool kNrm = false, class Probe = R32NoProbe>
inline bool fft32r_launch_one(const FftPlan &plan, const DirectParams &q, int nch, hipStream_t s, std::string &err,
                              FftNrm nrm = FftNrm{}) {
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(&fir_fft32r_kernel<kOut, kNrm, Probe>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kR32LdsBytes) == hipSuccess;
    }();
    (void)attr;
    const int64_t nseg = (q.end - q.seg0 + plan.B - 1) / plan.B;
    const int64_t units = nseg * nch; // < 2^31 (fft_launch)
    const int64_t grid = std::min<int64_t>(units, (int64_t)plan.cus);
    if constexpr (kNrm) {
        // whole 2 048-float blocks per unit (two halves of <= kNrmK32 x 1 024, fft_nrm_fusable)
        const int64_t per = (nrm.count + units - 1) / units;
        nrm.slice = (per + 2047) / 2048 * 2048;
        if (nrm.slice > (int64_t)kNrmK32 * 2048) {
            err = "normalize slice too large to fuse";
            return false;
        }
    }
    hipLaunchKernelGGL((fir_fft32r_kernel<kOut, kNrm, Probe>), dim3((unsigned)grid), dim3(kFftNT), kR32LdsBytes, s, q,
                       plan.d_pair, plan.d_tw, plan.d_task, plan.B, fft_grid(nseg, units), plan.c8[0].x, nrm);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        err = hipGetErrorString(e);
        return false;
    }
    return true;
}

template <int kOut>
inline bool fft32_launch_one(const FftPlan &plan, const DirectParams &q, int part, int nch, hipStream_t s,
                             std::string &err) {
    if constexpr (kOut == kFftOutSym)
        if (plan.reg32) return fft32r_launch_one<kOut>(plan, q, nch, s, err);
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(&fir_fft32_f64_kernel<kOut>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)fft_lds_bytes(kFft32L)) == hipSuccess;
    }();
    (void)attr;
    const int64_t nseg = (q.end - q.seg0 + plan.B - 1) / plan.B;
    const int64_t units = nseg * nch; // < 2^31 (fft_launch)
    const int64_t grid = std::min<int64_t>(units, (int64_t)plan.cus); // one 145 KiB workgroup per CU
    if (!q.park && kParkSlab > 0) {
        err = "L = 32768 launch without its park slab";
        return false;
    }
    hipLaunchKernelGGL((fir_fft32_f64_kernel<kOut>), dim3((unsigned)grid), dim3(kFftNT), fft_lds_bytes(kFft32L), s,
                       q, plan.d_pair + (size_t)part * 2 * kFftPairTable, plan.d_tw, plan.d_task, plan.B,
                       fft_grid(nseg, units), plan.c8[(size_t)part]);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        err = hipGetErrorString(e);
        return false;
    }
    return true;
}

template <int kOut, bool kNrm = false>
inline bool fft_launch_one(const FftPlan &plan, const DirectParams &q, int part, int nch, hipStream_t s,
                           std::string &err, FftNrm nrm = FftNrm{}) {
    if constexpr (kOut == kFftOutSym)
        if (plan.reg32) return fft32r_launch_one<kOut, kNrm>(plan, q, nch, s, err, nrm);
    if constexpr (!kNrm)
        if (plan.L == kFft32L) return fft32_launch_one<kOut>(plan, q, part, nch, s, err);
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(&fir_fft_f64_kernel<kOut, kNrm>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)fft_lds_bytes()) == hipSuccess;
    }();
    (void)attr;
    const int64_t nseg = (q.end - q.seg0 + plan.B - 1) / plan.B;
    const int64_t units = nseg * nch; // < 2^31 (fft_launch)
    const int64_t grid = std::min<int64_t>(units, (int64_t)plan.cus); // one 137 KiB workgroup per CU
    const FftGrid gd = fft_grid(nseg, units);
    if constexpr (kNrm) {
        // the previous file's floats over this launch's units, whole 1 024-float
        // blocks, at most kNrmK per thread (fft_nrm_fits)
        const int64_t per = (nrm.count + units - 1) / units;
        nrm.slice = (per + 1023) / 1024 * 1024;
        if (nrm.slice > (int64_t)kNrmK * 1024) {
            err = "normalize slice too large to fuse";
            return false;
        }
        hipLaunchKernelGGL((fir_fft_f64_kernel<kOut, true>), dim3((unsigned)grid), dim3(kFftNT), fft_lds_bytes(),
                           s, q, plan.d_pair + (size_t)part * kFftPairTable, plan.d_tw, plan.d_task, plan.B, gd,
                           plan.c8[(size_t)part], nrm);
    } else
        hipLaunchKernelGGL((fir_fft_f64_kernel<kOut, false>), dim3((unsigned)grid), dim3(kFftNT), fft_lds_bytes(),
                           s, q, plan.d_pair + (size_t)part * kFftPairTable, plan.d_tw, plan.d_task, plan.B, gd,
                           plan.c8[(size_t)part], FftNrm{});
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        err = hipGetErrorString(e);
        return false;
    }
    return true;
}

// Partitioned filters (plan.parts > 1) keep f64 partial sums: 2^26 outputs
// per chunk keep the scratch's byte offsets inside the 32-bit buffer range.
inline int64_t fft_chunk_outputs(const FftPlan &plan) {
    return plan.parts == 1 ? fft_chunk(plan) : std::min<int64_t>(fft_chunk(plan), (int64_t)1 << 26);
}
// The segment grid is anchored at output 0 of the channel: segment s covers
// outputs [s B, (s + 1) B) whatever range a call asks for, and launch chunks
// are whole segments.  A unit's outputs depend only on the samples it reads,
// so every output comes out the same, bit for bit, from any call whose input
// window holds its unit's samples (fft_window): the whole-channel call,
// windowed calls over any sub-range, chunked launches and channel groups all
// agree.  That is FilterCore.h's partition invariance -- ProcessFile.cp:60-83
// splits a channel into per-thread ranges and the result does not depend on
// how -- kept by the FFT method.  A range that starts inside a segment pays
// for that whole segment (at most one extra unit per channel and call).
inline int64_t fft_grid_start(const FftPlan &plan, int64_t start) { return start - start % plan.B; }
inline int64_t fft_chunk_span(const FftPlan &plan) {
    return std::max<int64_t>(plan.B, fft_chunk_outputs(plan) / plan.B * plan.B);
}
// Input samples [lo, hi) the units of outputs [start, end) read (unclipped;
// samples outside the channel are zeros to every unit alike).  Segment n0 of
// partition k reads x[n0 - half + k ntaps_k + i], i < L.
inline void fft_window(const FftPlan &plan, int64_t half, int64_t start, int64_t end, int64_t &lo, int64_t &hi) {
    const int64_t g0 = fft_grid_start(plan, start);
    const int64_t last = g0 + std::max<int64_t>(0, (end - g0 + plan.B - 1) / plan.B - 1) * plan.B;
    lo = g0 - half;
    hi = last - half + (int64_t)(plan.parts - 1) * plan.ntaps + plan.L;
}
// Segments of the first launch chunk of [p.start, p.end)
inline int64_t fft_first_nseg(const FftPlan &plan, const DirectParams &p) {
    const int64_t g0 = fft_grid_start(plan, p.start);
    return (std::min(p.end - g0, fft_chunk_span(plan)) + plan.B - 1) / plan.B;
}
// Doubles of partial-sum scratch one fft_launch of p over nch channels needs
// (0 for a single-partition filter); the chunks reuse it in stream order.
inline size_t fft_scratch_doubles(const FftPlan &plan, const DirectParams &p, int nch) {
    if (plan.parts == 1 || p.end <= p.start) return 0;
    return (size_t)std::min<int64_t>(p.end - p.start, fft_chunk_span(plan)) * (size_t)std::max(nch, 1);
}
// Doubles of park slab an L = 32768 launch needs (one slab per workgroup of
// the persistent grid, fir_fft32.hpp); launches on one stream reuse it.
inline size_t fft32_park_doubles(const FftPlan &plan) {
    return plan.L == kFft32L && !plan.reg32 ? (size_t)plan.cus * kParkSlab * kFftNT * 2 : 0;
}

// Filter outputs [p.start, p.end) of nch channels.  p.half / p.ntaps are the
// filter's own (the plan holds the partitioning); a partitioned filter needs
// p.y64 = fft_scratch_doubles() of scratch, owned by the caller's stream.
// Largest unit count of one launch: 2^31 - 1 (FftGrid's 32-bit unit index);
// FftTuning::max_units lowers it (tests exercise the channel-group split with
// small values)
inline int64_t fft_max_units(const FftPlan &plan) {
    const int64_t m = plan.tune.max_units;
    return m >= 1 && m < ((int64_t)1 << 31) ? m : (((int64_t)1 << 31) - 1);
}
inline bool fft_launch_group(const FftPlan &plan, const DirectParams &p, int nch, hipStream_t s,
                             std::string &err, const FftNrm *nrm);
// Can fft_launch carry a previous file's normalize (FftNrm) in its first
// launch?  Single-partition filters on the L = 16 384 or the register-resident
// L = 32 768 kernel, 16-B aligned buffer; otherwise the caller runs the
// normalize pass itself.  The first launch (the one that carries it) must
// spread the previous file's floats at <= kNrmK x 1 024 per unit (kNrmK32 x
// 2 048 on the register kernel: two halves).
// Floats of a previous file one unit of the plan's kernel rescales at most
// (0: the kernel carries none): kNrmK blocks of 1 024 on the L = 16 384
// kernel, two halves of kNrmK32 blocks on the register kernel.  Exported as
// lcfir_ctx_fft_units' nrm_floats (tests size the fused / separate switch
// from it).
inline int64_t fft_nrm_unit_floats(const FftPlan &plan) {
    if (plan.parts != 1) return 0;
    if (plan.reg32) return (int64_t)kNrmK32 * 2048;
    return plan.L == kFftL ? (int64_t)kNrmK * 1024 : 0;
}
inline bool fft_nrm_fusable(const FftPlan &plan, const FftNrm &nrm, const DirectParams &p, int nch) {
    const int64_t cap = fft_nrm_unit_floats(plan);
    if (cap == 0 || !nrm.y || !nrm.peak || nrm.npeak < 1 || (reinterpret_cast<uintptr_t>(nrm.y) & 15) != 0 ||
        p.end <= p.start || nch <= 0)
        return false;
    const int64_t nseg = fft_first_nseg(plan, p);
    const int64_t group = std::max<int64_t>(1, std::min<int64_t>(nch, fft_max_units(plan) / nseg));
    const int64_t units = nseg * group;
    const int64_t per = (nrm.count + units - 1) / units;
    // whole blocks per unit: 2 048 floats on the register kernel (two halves), 1 024 otherwise
    const int64_t blk = plan.reg32 ? 2048 : 1024;
    return (per + blk - 1) / blk * blk <= cap;
}
// nrm: a previous file's normalize to fuse (fft_nrm_fusable must hold), or null
inline bool fft_launch(const FftPlan &plan, const DirectParams &p, int nch, hipStream_t s,
                       std::string &err, const FftNrm *nrm = nullptr) {
    if (p.end - p.start <= 0 || nch <= 0) return true;
    if (nch > 65535) {
        err = "too many channels for one launch";
        return false;
    }
    if (plan.parts > 1 && !p.y64) {
        err = "partitioned filter without partial-sum scratch";
        return false;
    }
    // the kernels index units in 32 bits (FftGrid): channel groups keep every
    // launch's channels x segments below 2^31 (the partial-sum scratch is
    // reused by each group in stream order)
    const int64_t nseg = fft_first_nseg(plan, p);
    const int group = (int)std::max<int64_t>(1, std::min<int64_t>(nch, fft_max_units(plan) / nseg));
    for (int c0 = 0; c0 < nch; c0 += group) {
        DirectParams q = p;
        q.x = p.x + (int64_t)c0 * p.x_stride;
        q.y = p.y + (int64_t)c0 * p.y_stride;
        if (p.peak) q.peak = p.peak + (int64_t)c0 * p.peak_stride;
        if (!fft_launch_group(plan, q, std::min(group, nch - c0), s, err, c0 == 0 ? nrm : nullptr)) return false;
    }
    return true;
}
inline bool fft_launch_group(const FftPlan &plan, const DirectParams &p, int nch, hipStream_t s,
                             std::string &err, const FftNrm *nrm) {
    const int64_t span = fft_chunk_span(plan);
    const int64_t g0 = fft_grid_start(plan, p.start);
    for (int64_t cs = g0; cs < p.end; cs += span) {
        DirectParams q = p;
        q.seg0 = cs;
        q.start = std::max(cs, p.start);
        q.end = std::min(p.end, cs + span);
        // every partition of every unit reads inside fft_window
        int64_t wlo, whi;
        fft_window(plan, p.half, q.start, q.end, wlo, whi);
        const int64_t lo = std::max(p.x_lo, wlo);
        const int64_t hi = std::max(lo, std::min(p.x_hi, whi));
        q.x = p.x + (lo - p.x_lo);
        q.x_lo = lo;
        q.x_hi = hi;
        q.ntaps = plan.ntaps;
        if (plan.parts == 1) {
            // the first chunk's launch carries the fused normalize
            const bool fuse = nrm && cs == g0;
            bool ok;
            if (plan.sym)
                ok = fuse ? fft_launch_one<kFftOutSym, true>(plan, q, 0, nch, s, err, *nrm)
                          : fft_launch_one<kFftOutSym>(plan, q, 0, nch, s, err);
            else
                ok = fuse ? fft_launch_one<kFftOutF32, true>(plan, q, 0, nch, s, err, *nrm)
                          : fft_launch_one<kFftOutF32>(plan, q, 0, nch, s, err);
            if (!ok) return false;
            continue;
        }
        // the caller's scratch (p.y64, fft_scratch_doubles): f64 partial sums of
        // this chunk, element 0 = output q.start
        q.y64 = p.y64;
        q.y64_stride = q.end - q.start;
        for (int part = 0; part < plan.parts; ++part) {
            DirectParams qp = q;
            qp.half = p.half - part * plan.ntaps; // partition part covers taps [part * ntaps, ...)
            qp.peak = part == plan.parts - 1 ? p.peak : nullptr;
            bool ok;
            if (part == 0) ok = fft_launch_one<kFftOutFirst>(plan, qp, part, nch, s, err);
            else if (part < plan.parts - 1) ok = fft_launch_one<kFftOutAdd>(plan, qp, part, nch, s, err);
            else ok = fft_launch_one<kFftOutLast>(plan, qp, part, nch, s, err);
            if (!ok) return false;
        }
    }
    return true;
}

// stream-ordered on s (the plan was built on it); the caller syncs s
inline void fft_plan_free(FftPlan &plan, hipStream_t s) {
    if (plan.d_pair) (void)hipFreeAsync(plan.d_pair, s);
    if (plan.d_tw) (void)hipFreeAsync(plan.d_tw, s);
    if (plan.d_task) (void)hipFreeAsync(plan.d_task, s);
    plan = FftPlan{};
}

} // namespace lcfir

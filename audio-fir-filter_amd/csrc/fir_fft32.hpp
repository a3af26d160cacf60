// fir_fft32.hpp -- the L = 32 768 overlap-save segment for long filters.
//
// Same contract as fir_fft_f64_kernel (fir_fft.hpp), with segments twice as
// long: B = L - T + 1 outputs per segment, so at T = 8 001 a segment keeps 76 %
// of its transform instead of 51 %, and filters up to 30 721 taps need no
// partitions (config 1's 19 201 taps: one pass instead of two).
//
// The 16 384-point complex transform of a segment (z[m] = x[2m] + i x[2m+1])
// does not fit the 160 KiB LDS (256 KiB of f64 complex), so it is split by
// the parity of its bins (radix-2 decimation in frequency) into two
// 8192-point transforms that take turns in the 128 KiB work array:
//
//   half E: Z[2 kappa]     = FFT_8192(z[m] + z[m + 8192])[kappa]
//   half O: Z[2 kappa + 1] = FFT_8192((z[m] - z[m + 8192]) W_16384^m)[kappa]
//
// Bins k and M - k share a parity, so the real split + filter multiply +
// merge (the pair step) stays inside a half: half E pairs kappa <-> 8192 -
// kappa (fir_fft.hpp's lane structure, special lane included), half O pairs
// kappa <-> 8191 - kappa (columns w and 15 - w in every wave, task B the mirror
// of task A: no self-paired bins).  Each half's column phase is fir_fft.hpp's
// fft_columns.  With m = 512 a + b (thread b, register a):
//   stage 1 (thread b): u_a = z_a + z_{a+16}, d_a = z_a - z_{a+16}; 16-point
//     DFTs; half E times W_8192^(b c) into LDS, half O times W_32^a (register
//     constants) and W_16384^b W_8192^(b c) parked in registers;
//   half E's columns; swap: thread b reads its 16 half-E inverse columns and
//     writes its parked half-O values to the same addresses; half E's final
//     16-point DFTs (W_8192^(b c)) are parked instead;
//   half O's columns; final: half O's 16-point DFTs (W_16384^b W_8192^(b c)),
//     times W_32^a, and the radix-2 merge
//       out[m] = E[m] + O'[m],  out[m + 8192] = E[m] - O'[m]
//     then c[2m] = Re out[m], c[2m+1] = -Im out[m] as in fir_fft.hpp.
// Per segment: 4 workgroup barriers and 12 LDS round trips of the work array
// (2 and 6 per L = 16 384 segment: the same per transform point).
//
// Where the parked half lives.  It is 16 complex f64 per thread (64 VGPRs),
// and fft_columns alone already needs ~190 of the 256 VGPRs two waves per SIMD
// allow (kParkRegs = 16 measured 252 spilled VGPRs at compile time).  So
// kParkRegs of the 16 stay in registers and the rest go to a per-workgroup
// slab of global memory (p.park: [workgroup][16 - kParkRegs][512] double2,
// coalesced b128 stores and loads), written right after they are computed and
// read back just before the barrier that precedes their use, so the loads
// are in flight while the waves wait.  The slab is reused every segment
// (2 x 128 KiB of traffic per workgroup and segment at kParkRegs = 0,
// normally L2 / Infinity Cache hits).  scripts/fft32_model.py is the numpy
// model of this flow (index maps, pair tables, merge), checked against direct
// convolution.
//
// Included by fir_fft.hpp after its device helpers, inside namespace lcfir.

constexpr int kFft32L = 32768;
// parked values per thread kept in registers (the rest in DirectParams::park)
constexpr int kParkRegs = 0;
constexpr int kParkSlab = 16 - kParkRegs; // double2 per thread in the slab
// LDS twiddles: W_8192^i (i < 512), W_512^i (i < 64, fft_columns), W_16384^i (i < 512)
constexpr int kFft32Tw = 512 + 64 + 512;
constexpr int kFft32TwOdd = 576;

// LDS slot of half O's column c: wave w owns c = w and 15 - w in slots 2w, 2w + 1
__host__ __device__ constexpr int fft32_slot_odd(int c) { return c < 8 ? 2 * c : 31 - 2 * c; }
constexpr int fft32_slot_odd_column(int s) { return (s & 1) ? (31 - s) / 2 : s / 2; }

// Half O's task word of thread t = 64 w + lane: task A = (w, lane & 7, lane >> 3),
// task B = (15 - w, 7 - d1, 7 - e1); bins kappa = c + 16 (d1 + 8 e1 + 64 e2) and
// 8191 - kappa share the lane (A[e2] <-> B[7 - e2]).
inline uint32_t fft32_task_word_odd(int t) {
    const int w = t >> 6, lane = t & 63;
    const int ca = w, cb = 15 - w, da = lane & 7, ea = lane >> 3, db = 7 - da, eb = 7 - ea;
    return (uint32_t)(fft32_slot_odd(ca) | da << 4 | ea << 7 | fft32_slot_odd(cb) << 10 | db << 14 | eb << 17);
}

// W_32^r = cos(pi r / 16) - i sin(pi r / 16), r < 16
constexpr double kW32[16][2] = {
    {1.0, 0.0},
    {0.98078528040323044913, -0.19509032201612826785},
    {0.92387953251128675613, -0.38268343236508977173},
    {0.83146961230254523708, -0.55557023301960222474},
    {0.70710678118654752440, -0.70710678118654752440},
    {0.55557023301960222474, -0.83146961230254523708},
    {0.38268343236508977173, -0.92387953251128675613},
    {0.19509032201612826785, -0.98078528040323044913},
    {0.0, -1.0},
    {-0.19509032201612826785, -0.98078528040323044913},
    {-0.38268343236508977173, -0.92387953251128675613},
    {-0.55557023301960222474, -0.83146961230254523708},
    {-0.70710678118654752440, -0.70710678118654752440},
    {-0.83146961230254523708, -0.55557023301960222474},
    {-0.92387953251128675613, -0.38268343236508977173},
    {-0.98078528040323044913, -0.19509032201612826785}};

// a * W_32^r for a compile-time r (after unrolling): free for r = 0 and 8
__device__ __forceinline__ double2 w32mul(double2 a, int r) {
    if (r == 0) return a;
    if (r == 8) return mul_mi(a);
    return cmul(a, make_double2(kW32[r][0], kW32[r][1]));
}

// Output stage of one unit: outputs c[2m], c[2m+1] (m = j + 512 r, r < 32) of
// X(r) = E[r] + O[r] (r < 16) or E[r-16] - O[r-16], as fir_fft_f64_kernel's
// stores (range-checked buffer resources, nt stores, fused peak, partitioned
// modes).  Returns this lane's max |y| over the unit.
template <int kOut>
__device__ __forceinline__ float fft32_store_unit(const DirectParams &p, int ch, int64_t n0, int B, int j,
                                                  const double2 (&E)[16], const double2 (&O)[16]) {
    constexpr bool kSym = kOut == kFftOutSym;
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const __amdgpu_buffer_rsrc_t ys =
        __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
    // valid outputs c in [cmin, cmax): [T-1, L) causal, [half, L - half) zero-phase
    const int cmin = kSym ? p.half : p.ntaps - 1;
    const int cmax = kSym ? kFft32L - p.half : kFft32L;
    const int64_t off = n0 - cmin - p.start; // offset (samples) of c[0] from start
    const int64_t oend = p.end - p.start;
    float pk = 0.0f;
    auto X = [&](int r) -> double2 { return r < 16 ? cadd(E[r], O[r]) : csub(E[r - 16], O[r - 16]); };
    if constexpr (kOut == kFftOutF32 || kSym) {
        if (n0 >= p.start && n0 + B <= p.end) {
            // every output of the unit is in [start, end): the pair (c, c+1) is
            // valid iff cmin <= c < cmax; both stores share one offset
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const int c = 2 * (j + 512 * r);
                const double2 x = X(r);
                const float f0 = (float)x.x, f1 = (float)(-x.y);
                const bool ok = c >= cmin && (!kSym || c < cmax);
                const int ob = ok ? (int)((off + c) * 4) : (int)0x80000000;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ob, 0, kNtStore);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ob + 4, 0, kNtStore);
                pk = fmaxf(pk, ok ? fmaxf(fabsf(f0), fabsf(f1)) : 0.0f);
            }
        } else {
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const int c = 2 * (j + 512 * r);
                const double2 x = X(r);
                const float f0 = (float)x.x, f1 = (float)(-x.y);
                const int64_t o = off + c;
                const bool ok0 = c >= cmin && c < cmax && o >= 0 && o < oend,
                           ok1 = c + 1 >= cmin && c + 1 < cmax && o + 1 >= 0 && o + 1 < oend;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(o * 4) : (int)0x80000000,
                                                      0, kNtStore);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                      ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, kNtStore);
                pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
            }
        }
    } else {
        // partitioned filter: f64 partial sums in p.y64 (fir_fft_f64_kernel)
        double *zb = p.y64 + (int64_t)ch * p.y64_stride;
        const __amdgpu_buffer_rsrc_t zs = __builtin_amdgcn_make_buffer_rsrc(zb, (short)0, (int)(oend * 8), 0x00020000);
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const int c = 2 * (j + 512 * r);
            const double2 x = X(r);
            const int64_t o = off + c;
            const bool ok0 = c >= cmin && o >= 0 && o < oend, ok1 = c + 1 >= cmin && o + 1 >= 0 && o + 1 < oend;
            const int oz0 = ok0 ? (int)(o * 8) : (int)0x80000000;
            const int oz1 = ok1 ? (int)(o * 8 + 8) : (int)0x80000000;
            double v0 = x.x, v1 = -x.y;
            if constexpr (kOut != kFftOutFirst) {
                v0 += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zs, oz0, 0, 0));
                v1 += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zs, oz1, 0, 0));
            }
            if constexpr (kOut == kFftOutLast) {
                const float f0 = (float)v0, f1 = (float)v1;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(o * 4) : (int)0x80000000,
                                                      0, kNtStore);
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

// Persistent, XCD-aware grid as fir_fft_f64_kernel (one 512-thread workgroup
// per CU, fft_unit32).  pair: half E's table then half O's (kFftPairTable
// each, fir_fft.hpp's layouts); task: [2][512] task words (E, O); tw:
// kFft32Tw twiddles; c8: half E's special-lane bin-M/2 coefficient; p.park:
// gridDim.x x kParkSlab x 512 double2 of slab (fft32_park_doubles).
template <int kOut>
__global__ __launch_bounds__(kFftNT) void fir_fft32_f64_kernel(DirectParams p, const double2 *__restrict__ pair,
                                                              const double2 *__restrict__ tw,
                                                              const uint32_t *__restrict__ task, int B,
                                                              FftGrid gd, double2 c8) {
    extern __shared__ double2 flds[];
    double2 *twl = flds + kFftM; // the kFft32Tw twiddles, LDS-resident
    for (int i = threadIdx.x; i < kFft32Tw; i += kFftNT) twl[i] = tw[i];
    float2 v[32]; // samples of the unit about to start
    {
        const int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units);
        const int c = fft_div(u, gd);
        fft_load_unit<32>(p, c, p.seg0 + (int64_t)(u - c * gd.nseg) * B, threadIdx.x, v);
    }
    // every prefetch load retired at the loop head on both paths (fir_fft.hpp)
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    uint32_t tkE = task[threadIdx.x], tkO = task[kFftNT + threadIdx.x];
    asm volatile("" : "+v"(tkE), "+v"(tkO));
    const double2 *pairO = pair + kFftPairTable;
    float pk_run = 0.0f;
    int pk_ch = -1;
    float *pk_lds = reinterpret_cast<float *>(twl + kFft32Tw);
    int pk_pending = -1;
    int rnd = 0;
    for (int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units); u < gd.units;
         u = fft_unit32(++rnd, blockIdx.x, gridDim.x, gd.units)) {
        int j = threadIdx.x;
        asm volatile("" : "+v"(j));
        const int ch = fft_div(u, gd);
        const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;
        double2 park[16]; // the half that is not in LDS: O's stage-1 values, then E's outputs
        double2 *pb = p.park + (size_t)blockIdx.x * kParkSlab * kFftNT + j; // this thread's slab entries

        // ---- stage 1: the radix-2 split, both halves' 16-point DFTs (half E
        // first, into LDS; then half O from the same samples, parked)
        {
            double2 a[16];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                a[r] = make_double2((double)v[r].x + (double)v[r + 16].x, (double)v[r].y + (double)v[r + 16].y);
            dft16(a);
            twiddle16(a, twl[j]); // W_8192^(j c)
            // no barrier before this write: thread j rewrites the addresses it
            // read itself in the previous unit's final phase
#pragma unroll
            for (int c = 0; c < 16; ++c) flds[512 * fft_slot(c) + j] = a[c];
        }
        __builtin_amdgcn_sched_barrier(0);
        {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                park[r] = w32mul(make_double2((double)v[r].x - (double)v[r + 16].x,
                                              (double)v[r].y - (double)v[r + 16].y), r);
            dft16(park);
            const double2 w1 = twl[kFft32TwOdd + j]; // W_16384^j
#pragma unroll
            for (int r = 0; r < 16; ++r) park[r] = cmul(park[r], w1);
            twiddle16(park, twl[j]); // W_8192^(j c)
#pragma unroll
            for (int r = kParkRegs; r < 16; ++r) pb[(r - kParkRegs) * kFftNT] = park[r];
        }
        __syncthreads();
        if (pk_pending >= 0) {
            if (threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
            pk_pending = -1;
        }

        // ---- half E: the even bins (a fresh index: the column phase's
        // addresses die with it instead of living across both halves)
        {
            int jc = threadIdx.x;
            asm volatile("" : "+v"(jc));
            fft_columns<kOut, false>(flds, twl, pair, tkE, c8, false, jc, rnd, [] {});
        }
        // the parked half O values back, in flight across the barrier wait
#pragma unroll
        for (int r = kParkRegs; r < 16; ++r) park[r] = pb[(r - kParkRegs) * kFftNT];
        __syncthreads();

        // ---- swap: half E's inverse columns out of LDS, half O's stage-1 values in
        {
            double2 a[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) a[c] = flds[512 * fft_slot(c) + j];
#pragma unroll
            for (int c = 0; c < 16; ++c) flds[512 * fft32_slot_odd(c) + j] = park[c];
            twiddle16(a, twl[j]); // W_8192^(j c)
            dft16(a);
#pragma unroll
            for (int r = 0; r < 16; ++r) park[r] = a[r]; // E[j + 512 r]
#pragma unroll
            for (int r = kParkRegs; r < 16; ++r) pb[(r - kParkRegs) * kFftNT] = park[r];
        }
        __syncthreads();

        // ---- half O: the odd bins
        {
            int jc = threadIdx.x;
            asm volatile("" : "+v"(jc));
            fft_columns<kOut, false>(flds, twl, pairO, tkO, c8, true, jc, rnd, [] {});
        }
        // the next unit's samples (the last unit reloads itself): their
        // latency hides behind the barrier wait and the final phase
        {
            const int un1 = fft_unit32(rnd + 1, blockIdx.x, gridDim.x, gd.units);
            const int un = un1 < gd.units ? un1 : u;
            const int cn = fft_div(un, gd);
            fft_load_unit<32>(p, cn, p.seg0 + (int64_t)(un - cn * gd.nseg) * B, j, v);
        }
        // half E's outputs back from the slab, in flight across the barrier wait
#pragma unroll
        for (int r = kParkRegs; r < 16; ++r) park[r] = pb[(r - kParkRegs) * kFftNT];
        __syncthreads();

        // ---- final: half O's 16-point DFTs, W_32^a, the radix-2 merge, stores
        double2 a[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = flds[512 * fft32_slot_odd(c) + j];
        twiddle16(a, twl[j]); // W_8192^(j c)
        dft16(a);
        {
            const double2 w1 = twl[kFft32TwOdd + j]; // W_16384^j
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = w32mul(cmul(a[r], w1), r);
        }
        // the prefetch has had the barrier wait and the DFTs to land; waiting
        // here (not at the loop head) keeps the stores out of the wait
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
        const float pk = fft32_store_unit<kOut>(p, ch, n0, B, j, park, a);
        if (ch != pk_ch) {
            if (p.peak && pk_ch >= 0) {
                fft_peak_stage(pk_lds, pk_run);
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
        if (pk_pending >= 0 && threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
        __syncthreads();
        fft_peak_stage(pk_lds, pk_run);
        __syncthreads();
        if (threadIdx.x == 0) fft_peak_commit(p, pk_ch, pk_lds);
    }
}

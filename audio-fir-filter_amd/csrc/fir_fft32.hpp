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
// allow.  So kParkRegs of the 16 stay in registers (0 in the product: 2 fits
// the zero-phase form spill-free but measured no faster) and the rest go to a
// per-workgroup slab of global memory (p.park: [workgroup][16 - kParkRegs][512]
// double2, coalesced b128 stores and loads), written right after they are
// computed and read back just before the barrier that precedes their use, so
// the loads are in flight while the waves wait.  The slab is reused every
// segment (2 x 128 KiB of traffic per workgroup and segment, L2 / Infinity
// Cache hits).  scripts/fft32_model.py is the numpy model of this flow (index
// maps, pair tables, merge), checked against direct convolution.
//
// Registers, round 3.  The first build kept the next unit's 32 float2 of
// samples in VGPRs across the final phase (beside the merge's 2 x 64) and
// spilled 42-63 VGPRs; every spill reload is a vector-memory instruction whose
// vmcnt wait also waited for the slab stores issued before it, and the
// kernel ran 1.3x its instruction count's time (PMC: SQ_WAIT_ANY 2x the
// L = 16 384 kernel's).  Now the samples are staged in LDS by LDS-DMA
// (fft32_stage_samples) and the task words are laundered per unit: the
// zero-phase form holds 232 VGPRs with no spills, 23 % faster.  Measured
// against the L = 16 384 kernel (tools/fft32_trace.hip, CHANGELOG.md s4.2): a unit
// costs 2.9x an L = 16 384 unit, so at 8 001 taps (config 3) the two are even
// and from ~9 000 taps on, and above all where L = 16 384 needs partitions
// (12 001 .. 30 001 taps), the longer segment wins (2x at 12 001 .. 19 201).
// fft_choose_seg_len picks per filter from those costs.
//
// Included by fir_fft.hpp after its device helpers, inside namespace lcfir.

// Phase timestamps for tools/fft32_trace.hip (off in the product build):
// lane 0 of every wave of workgroups < 64 records s_memtime at each phase
// boundary of its 3rd unit (round 2).
#ifdef LCFIR_FFT32_TRACE
__device__ unsigned long long g_fft32_trace[64][8][16];
#define FFT32_STAMP(i)                                                                     \
    do {                                                                                   \
        if (blockIdx.x < 64 && rnd == 2 && (threadIdx.x & 63) == 0)                        \
            g_fft32_trace[blockIdx.x][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define FFT32_STAMP(i) \
    do {               \
    } while (0)
#endif

constexpr int kFft32L = 32768;
// parked values per thread kept in registers (the rest in DirectParams::park)
constexpr int kParkRegs = 0;
constexpr int kParkSlab = 16 - kParkRegs; // double2 per thread in the slab
constexpr int kFft32StoreAux = kNtStore; // output store cache policy
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
        if ((cmin & 3) == 0 && n0 >= p.start && n0 + B <= p.end) {
            // Every output of the unit is in [start, end) and cmin, cmax are
            // multiples of 4, so the quad c .. c + 3 (c = 2 (j + 512 r), j
            // even) is valid or invalid as a whole.  Lanes j and j ^ 1 trade
            // one pair per two groups (DPP quad_perm [1,0,3,2]): the even lane
            // stores group 2k's quad, the odd lane group 2k + 1's -- 16 stores
            // of 16 bytes instead of 32 of 8.  The stores of a unit leave in
            // one burst from every wave of the CU, and their issue, not the
            // bytes, bounds the burst (MI355X_MICROARCH.md, store tail).
            const bool odd = j & 1;
            const int jq = j & ~1;
            using b128_t = decltype(__builtin_amdgcn_raw_buffer_load_b128(ys, 0, 0, 0));
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double2 xa = X(2 * k), xb = X(2 * k + 1);
                const float a0 = (float)xa.x, a1 = (float)(-xa.y), b0 = (float)xb.x, b1 = (float)(-xb.y);
                const int ca = 2 * (j + 1024 * k), cb = ca + 1024;
                const bool oka = ca >= cmin && (!kSym || ca < cmax), okb = cb >= cmin && (!kSym || cb < cmax);
                pk = fmaxf(pk, fmaxf(oka ? fmaxf(fabsf(a0), fabsf(a1)) : 0.0f, okb ? fmaxf(fabsf(b0), fabsf(b1)) : 0.0f));
                const int s0 = __float_as_int(odd ? a0 : b0), s1 = __float_as_int(odd ? a1 : b1);
                const int r0 = __builtin_amdgcn_update_dpp(0, s0, 0xB1, 0xF, 0xF, false);
                const int r1 = __builtin_amdgcn_update_dpp(0, s1, 0xB1, 0xF, 0xF, false);
                int4 q;
                q.x = odd ? r0 : __float_as_int(a0);
                q.y = odd ? r1 : __float_as_int(a1);
                q.z = odd ? __float_as_int(b0) : r0;
                q.w = odd ? __float_as_int(b1) : r1;
                const int cq = 2 * (jq + 512 * (2 * k + (odd ? 1 : 0)));
                const bool okq = cq >= cmin && (!kSym || cq < cmax);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128_t, q), ys,
                                                       okq ? (int)((off + cq) * 4) : (int)0x80000000, 0, kFft32StoreAux);
            }
        } else if (n0 >= p.start && n0 + B <= p.end) {
            // every output of the unit is in [start, end); cmin is not a
            // multiple of 4 (an odd one -- the zero-phase form of an odd half
            // -- splits a pair at each end): each output of a pair checked on
            // its own, both stores from one offset
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const int c = 2 * (j + 512 * r);
                const double2 x = X(r);
                const float f0 = (float)x.x, f1 = (float)(-x.y);
                const bool ok0 = c >= cmin && (!kSym || c < cmax), ok1 = c + 1 >= cmin && (!kSym || c + 1 < cmax);
                const int ob = (int)((off + c) * 4);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? ob : (int)0x80000000, 0,
                                                      kFft32StoreAux);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ok1 ? ob + 4 : (int)0x80000000, 0,
                                                      kFft32StoreAux);
                pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
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
                                                      0, kFft32StoreAux);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                      ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, kFft32StoreAux);
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
                                                      0, kFft32StoreAux);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys,
                                                      ok1 ? (int)(o * 4 + 4) : (int)0x80000000, 0, kFft32StoreAux);
                pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
            } else {
                using b64_t = decltype(__builtin_amdgcn_raw_buffer_load_b64(zs, 0, 0, 0));
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(b64_t, v0), zs, oz0, 0, kFft32StoreAux);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(b64_t, v1), zs, oz1, 0, kFft32StoreAux);
            }
        }
    }
    return pk;
}

// The samples of the next unit are staged in LDS, not in registers.  The
// final phase frees, in every slot of the work array, the 1 KiB block wave w's
// own lanes read (flds[512 s + 64 w, + 64)); wave w refills those 16 KiB with
// the next unit's z[512 a + 64 w + i] (a < 32, i < 64) -- exactly what its
// lanes' stage 1 reads -- as float2 at fft32_zidx(a, w, i).  Interior units
// arrive by LDS-DMA (buffer_load_dwordx4 ... lds: 16 instructions per wave,
// no VGPRs, in flight across the DFTs and stores); edge units by fft_load_unit's
// range-checked register loads and 32 ds_write_b64.  No other wave touches the
// block between wave w's final-phase reads and its next stage-1 writes, so
// only the wave's own order matters (its LDS operations execute in issue order).
__device__ __forceinline__ int fft32_zidx(int a, int w, int i) { return 1024 * (a >> 1) + 128 * w + 64 * (a & 1) + i; }

typedef __attribute__((address_space(3))) void fft_lds_void;

// Stage unit (ch, n0)'s samples into wave w's blocks (the caller has retired
// the wave's reads of them: s_waitcnt lgkmcnt(0)).
__device__ __forceinline__ void fft32_stage_samples(const DirectParams &p, int ch, int64_t n0, int j,
                                                    double2 *flds) {
    const int w = j >> 6, lane = j & 63;
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const int64_t w0 = n0 - p.half - p.x_lo; // window start inside the loaded range
    float2 *fz = reinterpret_cast<float2 *>(flds);
    if (w0 >= 0 && w0 + kFft32L <= p.x_hi - p.x_lo) {
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(x), (short)0, (int)((p.x_hi - p.x_lo) * 4), 0x00020000);
        // instruction s, lane l: z[512 a + 64 w + 2k], z[.. + 1] with a = 2s + (l >> 5),
        // k = l & 31, i.e. the 16 bytes at 4 w0 + 8192 s + 4096 (l >> 5) + 512 w + 16 (l & 31),
        // into LDS byte 8192 s + 1024 w + 16 l (= fft32_zidx(a, w, 2k))
        const int vofs = 4096 * (lane >> 5) + 512 * w + 16 * (lane & 31);
        const int sofs = (int)(w0 * 4);
#pragma unroll
        for (int s = 0; s < 16; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (fft_lds_void *)(flds + 512 * s + 64 * w), 16, vofs,
                                                     sofs + 8192 * s, 0, 0);
    } else {
        float2 v[32];
        fft_load_unit<32>(p, ch, n0, j, v);
#pragma unroll
        for (int a = 0; a < 32; ++a) fz[fft32_zidx(a, w, lane)] = v[a];
    }
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
    {
        const int u = fft_unit32(0, blockIdx.x, gridDim.x, gd.units);
        const int c = fft_div(u, gd);
        fft32_stage_samples(p, c, p.seg0 + (int64_t)(u - c * gd.nseg) * B, threadIdx.x, flds);
    }
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    const uint32_t tkE = task[threadIdx.x], tkO = task[kFftNT + threadIdx.x];
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
        const int w = j >> 6, lane = j & 63;
        const int ch = fft_div(u, gd);
        const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;
        double2 park[16]; // the half that is not in LDS: O's stage-1 values, then E's outputs
        double2 *pb = p.park + (size_t)blockIdx.x * kParkSlab * kFftNT + j; // this thread's slab entries
        FFT32_STAMP(0);

        // ---- stage 1: the samples out of the LDS image (the previous unit's
        // final phase staged them), the radix-2 split, both halves' 16-point
        // DFTs (half E into LDS, half O to the slab)
        {
            // (the staging transfers retired before the previous unit's stores)
            const float2 *fz = reinterpret_cast<const float2 *>(flds);
            float2 v[32];
#pragma unroll
            for (int r = 0; r < 32; ++r) v[r] = fz[fft32_zidx(r, w, lane)];
            double2 a[16];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                a[r] = make_double2((double)v[r].x + (double)v[r + 16].x, (double)v[r].y + (double)v[r + 16].y);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                park[r] = w32mul(make_double2((double)v[r].x - (double)v[r + 16].x,
                                              (double)v[r].y - (double)v[r + 16].y), r);
            dft16(a);
            twiddle16(a, twl[j]); // W_8192^(j c)
            // every lane of the wave has read its samples (same wave, issue order)
#pragma unroll
            for (int c = 0; c < 16; ++c) flds[512 * fft_slot(c) + j] = a[c];
            dft16(park);
            const double2 w1 = twl[kFft32TwOdd + j]; // W_16384^j
#pragma unroll
            for (int r = 0; r < 16; ++r) park[r] = cmul(park[r], w1);
            twiddle16(park, twl[j]); // W_8192^(j c)
#pragma unroll
            for (int r = kParkRegs; r < 16; ++r) pb[(r - kParkRegs) * kFftNT] = park[r];
        }
        FFT32_STAMP(1);
        __syncthreads();
        FFT32_STAMP(2);
        if (pk_pending >= 0) {
            if (threadIdx.x == 0) fft_peak_commit(p, pk_pending, pk_lds);
            pk_pending = -1;
        }

        // ---- half E: the even bins (fresh indices: the column phase's
        // addresses die with it instead of living across both halves)
        {
            int jc = threadIdx.x;
            uint32_t tk = tkE;
            asm volatile("" : "+v"(jc), "+v"(tk));
            fft_columns<kOut, false>(flds, twl, pair, tk, c8, false, jc, rnd, [] {});
        }
        FFT32_STAMP(3);
        // the parked half O values back, in flight across the barrier wait
        // and the swap's first DFT
#pragma unroll
        for (int r = kParkRegs; r < 16; ++r) park[r] = pb[(r - kParkRegs) * kFftNT];
        __syncthreads();
        FFT32_STAMP(4);

        // ---- swap: half E's inverse columns out of LDS and through their
        // final 16-point DFTs, then half O's stage-1 values in (thread j's own
        // addresses: no barrier between the reads and the writes)
        {
            double2 a[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) a[c] = flds[512 * fft_slot(c) + j];
            twiddle16(a, twl[j]); // W_8192^(j c)
            dft16(a);
#pragma unroll
            for (int c = 0; c < 16; ++c) flds[512 * fft32_slot_odd(c) + j] = park[c];
#pragma unroll
            for (int r = 0; r < 16; ++r) park[r] = a[r]; // E[j + 512 r]
#pragma unroll
            for (int r = kParkRegs; r < 16; ++r) pb[(r - kParkRegs) * kFftNT] = park[r];
        }
        FFT32_STAMP(5);
        __syncthreads();
        FFT32_STAMP(6);

        // ---- half O: the odd bins
        {
            int jc = threadIdx.x;
            uint32_t tk = tkO;
            asm volatile("" : "+v"(jc), "+v"(tk));
            fft_columns<kOut, false>(flds, twl, pairO, tk, c8, true, jc, rnd, [] {});
        }
        FFT32_STAMP(7);
        // half E's outputs back from the slab, in flight across the barrier wait
#pragma unroll
        for (int r = kParkRegs; r < 16; ++r) park[r] = pb[(r - kParkRegs) * kFftNT];
        __syncthreads();
        FFT32_STAMP(8);

        // ---- final: half O's columns out of LDS; the next unit's samples
        // into the freed blocks (unconditional -- the last unit restages
        // itself -- so the waits below count the same instructions on every
        // path); half O's 16-point DFTs, W_32^a, the radix-2 merge, stores
        double2 a[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = flds[512 * fft32_slot_odd(c) + j];
        const double2 wj = twl[j], w1 = twl[kFft32TwOdd + j]; // W_8192^j, W_16384^j
        // vmcnt(0) lgkmcnt(0): the wave's reads of its blocks have retired, and
        // so have half E's slab reloads -- the compiler does not count LDS-DMA
        // in vmcnt, so a wait it placed for them after the transfers below
        // would also wait for the transfers
        __builtin_amdgcn_s_waitcnt(0x0070);
        {
            const int un1 = fft_unit32(rnd + 1, blockIdx.x, gridDim.x, gd.units);
            const int un = un1 < gd.units ? un1 : u;
            const int cn = fft_div(un, gd);
            fft32_stage_samples(p, cn, p.seg0 + (int64_t)(un - cn * gd.nseg) * B, j, flds);
        }
        FFT32_STAMP(9);
        twiddle16(a, wj); // W_8192^(j c)
        dft16(a);
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = w32mul(cmul(a[r], w1), r);
        // the staging transfers have had the DFTs to land; waiting here, not
        // at the loop head, keeps the output stores out of the wait (the
        // compiler neither counts LDS-DMA in vmcnt nor orders it before LDS
        // reads: this explicit wait is what stage 1's reads rely on)
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
        FFT32_STAMP(10);
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
        FFT32_STAMP(11);
    }
    // the last unit's restaging transfer must land before the LDS is released
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

// fir_fft16r.hpp -- the L = 16 384 zero-phase overlap-save unit held in the
// registers of a 256-thread workgroup, two workgroups per CU (DESIGN.md s4.2,
// "L = 16 384 in registers, two workgroups per CU").
//
// fir_fft32r.hpp holds an L = 32 768 unit in the registers of one 512-thread
// workgroup per CU.  Its six barriers keep all eight waves in the same phase,
// so the CU's LDS pipe (the exchanges) and its f64 VALU (the DFTs) take turns,
// and every CU moves its unit's samples and outputs in the same window.  Here
// a unit is half as long and a workgroup a quarter of the CU's threads: two
// workgroups share each CU (one wave of each per SIMD, 256 VGPRs each, half
// the LDS each), and nothing ties their phases together -- one exchanges
// while the other computes, and each loads its samples straight into
// registers at its own time.  The same arithmetic per transform point as
// fir_fft32r (DFT32 / DFT16 / anchored twiddle chains, the zero-phase pair
// step), 8 % more of it per output at 4 001 taps (B = 12 384 of 16 384).
//
//   z[m] = x_seg[2m] + i x_seg[2m+1], m = 256 n + b (thread b, register n),
//   b = 16 beta + gamma;   bins k = k1 + 32 kappa + 512 lambda.
//   stage 1 (thread b): DFT32 over n -> k1, * W_8192^(b k1)
//   T1 (workgroup, 2 rounds): lane (w, s, gamma) gathers beta = 0..15 of
//       column P = 4 w + s (pair A, round 1, registers 0..15) and of its
//       mirror 32 - P (pair B, round 2; column 16 for P = 0)
//   stage 2 (both pairs): DFT16 over beta -> kappa, * W_256^(gamma kappa)
//   T2 (16-lane groups, 2 rounds: kappa < 8, kappa >= 8): lane q of group s
//       gathers gamma for task R1 (column, kappa < 8) and R2, its mirror
//       (32 - column, 15 - kappa)
//   stage 3: DFT16 over gamma -> lambda;  pair step R1[i] <-> R2[15 - i]
//   (bins k and N - k), the zero-phase pair table; then stage 3, T2, stage 2,
//   T1 and stage 1 again in reverse (the inverse as conj(FFT(conj(V)))).
// Wave 0's lane 0 holds the self-paired bins 0 and N/2 (tasks (0, 0) and
// (0, 8)) and permutes its registers through LDS around the pair step, as
// fir_fft32r's special lane.  scripts/fft16r_model.py is the numpy model of
// this flow (every register index, LDS slot, task and table slot; bank
// conflicts); tests/test_fft32_tables.py runs it on the host's tables.
//
// Included by fir_fft.hpp after fir_fft32r.hpp, inside namespace lcfir.

constexpr int kR16NT = 256;            // threads per workgroup
constexpr int kR16L = 16384;           // real samples per unit
constexpr int kR16WgPerCu = 2;         // persistent grid: workgroups per CU
constexpr int kR16Work = 4 * kR32Rg;   // LDS work array (double2): one 17-KiB region per wave
constexpr int kR16TwB = 0;             // W_8192^b, b < 256
constexpr int kR16TwG = 256;           // W_256^g, g < 16
constexpr int kR16Tw = 256 + 16;
constexpr int kR16SpecialLane = 0;     // of wave 0
constexpr size_t kR16PairTable = (size_t)24 * kR16NT; // double2: (p1, q2) [16][256], (p2 even, p2 odd) [8][256]
constexpr int kR16PairStores = 32;     // one 8-byte store per register pair
// a previous file's normalize carried by the launch (FftNrm): up to kNrmK16
// blocks of 1 024 floats per unit, one float4 per thread and block
constexpr int kNrmK16 = 16;
// LDS: work array, twiddles, 4 peak slots (one double2 of room), the special lane's 32 double2
constexpr size_t kR16LdsBytes = sizeof(double2) * (size_t)(kR16Work + kR16Tw + 2 + 32);
static_assert(kR16WgPerCu * kR16LdsBytes <= 160 * 1024, "two workgroups per CU must fit the 160 KiB LDS");

// Column P's pair-B mirror (32 - P; 16 for P = 0) and the LDS home (wave,
// group) of the reader of column k1: P = k1 for k1 < 16, 32 - k1 above (0 for 16)
__host__ __device__ constexpr int r16_home(int k1) { return k1 < 16 ? k1 : (k1 == 16 ? 0 : 32 - k1); }
__host__ __device__ constexpr int r16_col_b(int P) { return P == 0 ? 16 : 32 - P; }

// Task word of thread t (host): T2's read tasks (pair, kappa mod 8) for R1
// (bits 0..3) and R2 (bits 4..7), scripts/fft16r_model.py's t2_tasks
inline uint32_t r16_task_word(int t) {
    const int w = t >> 6, s = (t >> 4) & 3, q = t & 15;
    int p1, k1, p2, k2;
    if (w == 0 && s == 0) {
        if (q == 0) { // the special lane: (0, 0) and (0, 8), each self-paired
            p1 = 0, k1 = 0, p2 = 0, k2 = 8;
        } else if (q < 8) {
            p1 = 0, k1 = q, p2 = 0, k2 = 16 - q;
        } else {
            p1 = 1, k1 = q - 8, p2 = 1, k2 = 23 - q;
        }
    } else if (q < 8) {
        p1 = 0, k1 = q, p2 = 1, k2 = 15 - q;
    } else {
        p1 = 1, k1 = q - 8, p2 = 0, k2 = 23 - q;
    }
    return (uint32_t)(p1 | (k1 & 7) << 1 | p2 << 4 | (k2 & 7) << 5);
}
// bins of thread t's R1 / R2 registers lambda = 0..15 (host; pair tables)
inline void r16_task_bins(int t, int (&bx)[16], int (&by)[16]) {
    const int w = t >> 6, s = (t >> 4) & 3, P = 4 * w + s;
    const uint32_t tk = r16_task_word(t);
    const int cA = (tk & 1) ? r16_col_b(P) : P, kA = (tk >> 1) & 7;
    const int cB = ((tk >> 4) & 1) ? r16_col_b(P) : P, kB = 8 + ((tk >> 5) & 7);
    for (int l = 0; l < 16; ++l) {
        bx[l] = cA + 32 * kA + 512 * l;
        by[l] = cB + 32 * kB + 512 * l;
    }
}

// Samples of unit (ch, n0): v[n] = (x_seg[2m], x_seg[2m+1]), m = 256 n + b,
// x_seg[i] = x[n0 - half + i], through a range-checked resource over the
// loaded window (fft_load_unit's rule: offsets outside it, "negative" ones
// included, read 0; edge units load dword by dword so a pair straddling the
// window start keeps its in-range sample).
__device__ __forceinline__ void r16_load_unit(const DirectParams &p, int ch, int64_t n0, int b, float2 (&v)[32]) {
    const float *x = p.x + (int64_t)ch * p.x_stride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(x), (short)0, (int)((p.x_hi - p.x_lo) * 4), 0x00020000);
    const int64_t w0 = n0 - p.half - p.x_lo;
    const int off0 = (int)(w0 * 4) + 8 * b; // may be negative
    if (w0 >= 0 && w0 + kR16L <= p.x_hi - p.x_lo) {
#pragma unroll
        for (int n = 0; n < 32; ++n)
            v[n] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off0 + 2048 * n, 0, 0));
    } else {
#pragma unroll
        for (int n = 0; n < 32; ++n) {
            const int off = off0 + 2048 * n;
            v[n].x = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, (int)0x80000000));
            v[n].y = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, (int)0x80000000));
        }
    }
}

// a unit whose outputs take the pair-store path (kR16PairStores per lane)
__device__ __forceinline__ bool r16_pair_path(const DirectParams &p, int64_t n0, int B) {
    return (p.half & 1) == 0 && n0 >= p.start && (p.end - n0 >= B || ((p.end - n0) & 1) == 0);
}

// Outputs of one unit: c[2m] = Re out[m], c[2m+1] = -Im out[m], m = b + 256 n,
// valid for c in [half, L - half).  Pair stores through a per-unit resource
// when half is even (the range check drops the halo), else one dword per
// output with explicit range checks (fir_fft32r.hpp's r32_store_unit).
__device__ __forceinline__ float r16_store_unit(const DirectParams &p, int ch, int64_t n0, int B, int b,
                                                const double2 (&o)[32]) {
    float *yb = p.y + (int64_t)ch * p.y_stride + (p.start - p.y_lo);
    const int cmin = p.half, cmax = kR16L - p.half;
    float pk = 0.0f;
    if (r16_pair_path(p, n0, B)) {
        const int nrec = 4 * (int)(p.end - n0 < B ? p.end - n0 : B);
        const __amdgpu_buffer_rsrc_t yu =
            __builtin_amdgcn_make_buffer_rsrc(yb + (n0 - p.start), (short)0, nrec, 0x00020000);
        const int v0 = 8 * b - 4 * cmin;
        using b64_t = decltype(__builtin_amdgcn_raw_buffer_load_b64(yu, 0, 0, 0));
#pragma unroll
        for (int n = 0; n < kR16PairStores; ++n) {
            const float f0 = (float)o[n].x, f1 = (float)(-o[n].y);
            const int vo = v0 + 2048 * n;
            const float m = fmaxf(fabsf(f0), fabsf(f1));
            pk = (unsigned)vo < (unsigned)nrec ? fmaxf(pk, m) : pk;
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(b64_t, make_int2(__float_as_int(f0), __float_as_int(f1))), yu, vo, 0, kNtStore);
        }
    } else {
        const __amdgpu_buffer_rsrc_t ys =
            __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, (int)((p.end - p.start) * 4), 0x00020000);
        const int64_t off = n0 - cmin - p.start;
        const int64_t oend = p.end - p.start;
#pragma unroll
        for (int n = 0; n < 32; ++n) {
            const int c = 2 * (b + 256 * n);
            const float f0 = (float)o[n].x, f1 = (float)(-o[n].y);
            const int64_t oo = off + c;
            const bool ok0 = c >= cmin && c < cmax && oo >= 0 && oo < oend,
                       ok1 = c + 1 >= cmin && c + 1 < cmax && oo + 1 >= 0 && oo + 1 < oend;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f0), ys, ok0 ? (int)(oo * 4) : (int)0x80000000, 0,
                                                  kNtStore);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(f1), ys, ok1 ? (int)(oo * 4 + 4) : (int)0x80000000,
                                                  0, kNtStore);
            pk = fmaxf(pk, fmaxf(ok0 ? fabsf(f0) : 0.0f, ok1 ? fabsf(f1) : 0.0f));
        }
    }
    return pk;
}

// the wave's running peak into its LDS slot (uniform address), and thread 0's
// fold of the four slots into one atomicMax after the next barrier
__device__ __forceinline__ void r16_peak_stage(float *pk_lds, float pk) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) pk = fmaxf(pk, __shfl_xor(pk, s, 64));
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if ((threadIdx.x & 63) == 0) pk_lds[wv] = pk;
}
__device__ __forceinline__ void r16_peak_commit(const DirectParams &p, int ch, const float *pk_lds) {
    const float pk = fmaxf(fmaxf(pk_lds[0], pk_lds[1]), fmaxf(pk_lds[2], pk_lds[3]));
    atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(pk));
}

// Persistent, XCD-aware grid of kR16WgPerCu 256-thread workgroups per CU
// (fft_unit32), zero-phase single-partition filters (kFftOutSym).  pair:
// kR16PairTable (r16_plan_tables); tw: kR16Tw twiddles; task: 256
// r16_task_word; c8: the special lane's bin-N/2 coefficient (real).
// kNrm: the launch also rescales a previous file's outputs (FftNrm, the
// normalize_kernel rule): unit u takes floats [u slice, (u + 1) slice), loaded
// with the unit's samples and stored before its stage 1 -- the other
// workgroup on the CU computes through the loads' latency.
template <int kOut = kFftOutSym, bool kNrm = false, class Probe = R32NoProbe> // host-only users emit no stub
__global__ __launch_bounds__(kR16NT, 2) void fir_fft16r_kernel(DirectParams p, const double2 *__restrict__ pair,
                                                              const double2 *__restrict__ tw,
                                                              const uint32_t *__restrict__ task, int B, FftGrid gd,
                                                              double c8, FftNrm nrm) {
    extern __shared__ double2 flds[];
    bool nrm_on = false;
    double nrm_gain = 1.0;
    if constexpr (kNrm) {
        float pkv = 0.0f;
        for (int i = 0; i < nrm.npeak; ++i) pkv = fmaxf(pkv, __uint_as_float(nrm.peak[i]));
        nrm_on = (pkv > 1.0f || nrm.force) && pkv > 0.0f;
        nrm_gain = 1.0 / (double)pkv;
    }
    double2 *twl = flds + kR16Work; // kR16Tw twiddles, then 4 f32 peak slots, then the special lane's scratch
    for (int i = threadIdx.x; i < kR16Tw; i += kR16NT) twl[i] = tw[i];
    float *pk_lds = reinterpret_cast<float *>(twl + kR16Tw);
    double2 *spl = twl + kR16Tw + 2;
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
        const int ch = fft_div(u, gd);
        const int64_t n0 = p.seg0 + (int64_t)(u - ch * gd.nseg) * B;
        double2 a[32];
        Probe::stamp(0, rnd);
        // ---- stage 1: the samples straight into registers; DFT32; W_8192^(b k1)
        {
            float2 v[32];
            r16_load_unit(p, ch, n0, j, v);
            if constexpr (kNrm) {
                // the unit's normalize slice: loaded behind the samples, rescaled and
                // stored before stage 1 (an inactive launch loads through an empty
                // resource: no traffic, nothing stored)
                float4 nv[kNrmK16];
                fft_nrm_load<kNrmK16>(nrm, u, j, nrm_on, nv);
                if (nrm_on) fft_nrm_store<kNrmK16>(nrm, u, j, nrm_gain, nv);
            }
#pragma unroll
            for (int n = 0; n < 32; ++n) a[n] = make_double2((double)v[n].x, (double)v[n].y);
        }
        Probe::stamp(1, rnd);
        dft32(a);
        r32_chain32acc(a, twl[kR16TwB + j]);
        Probe::stamp(2, rnd);
        // ---- T1 round 1: registers 0..15 into the wave's own region (row k1)
#pragma unroll
        for (int i = 0; i < 16; ++i) flds[kR32Rg * w + 64 * i + lane] = a[i];
        r32_bar();
        Probe::stamp(3, rnd);
        if (pk_pending >= 0) {
            if (threadIdx.x == 0) r16_peak_commit(p, pk_pending, pk_lds);
            pk_pending = -1;
        }
        const int s = lane >> 4, gam = lane & 15;
        const int P = 4 * w + s;
        double2 c[32]; // c[0..15]: pair A (column P), c[16..31]: pair B (column r16_col_b(P))
        {
            // beta = i: thread 16 i + gam, row P (wave i >> 2)
            const int base = 64 * P + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) c[i] = flds[base + kR32Rg * (i >> 2) + 16 * (i & 3)];
        }
        Probe::stamp(4, rnd);
        r32_bar();
        // ---- T1 round 2: registers 16..31 into the region of their column's
        // reader (destination-major: row = the reader's group, slot = thread)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int home = r16_home(16 + i); // uniform: 4 wave + group of the column's reader
            flds[kR32Rg * (home >> 2) + 256 * (home & 3) + j] = a[16 + i];
        }
        r32_bar();
        Probe::stamp(5, rnd);
        {
            const int base = kR32Rg * w + 256 * s + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) c[16 + i] = flds[base + 16 * i];
        }
        Probe::stamp(6, rnd);
        // ---- stage 2: DFT16 over beta, * W_256^(gam kappa), both pairs
        double2 wg = twl[kR16TwG + gam];
        {
            double2 cA[16], cB[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                cA[i] = c[i];
                cB[i] = c[16 + i];
            }
            dft16f(cA);
            dft16f(cB);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                c[i] = cA[i];
                c[16 + i] = cB[i];
            }
        }
        {
            const double2 w2 = cmul(wg, wg);
            const double2 w4 = cmul(w2, w2);
            const double2 one = make_double2(1.0, 0.0);
            r32_chain_anchored<16>(c, 0, one, wg, w4);
            r32_chain_anchored<16>(c, 16, one, wg, w4);
        }
        Probe::stamp(7, rnd);
        // ---- the pair table's first half, in flight across T2
        double2 pq[16], p2v[8];
        {
            const double2 *pt = pair + j;
#pragma unroll
            for (int i = 0; i < 8; ++i) pq[i] = pt[kR16NT * i];
#pragma unroll
            for (int m = 0; m < 4; ++m) p2v[m] = pt[kR16NT * (16 + m)];
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- T2: two wave-local rounds (kappa < 8, kappa >= 8) in the wave's
        // region; rows of kR32Row slots: (group s, pair, kappa mod 8) x gamma
        uint32_t tk = tk_all;
        asm volatile("" : "+v"(tk)); // per unit: T2's addresses are not hoisted out of the loop
        const int rb1 = kR32Rg * w + 272 * s + 136 * (tk & 1) + kR32Row * ((tk >> 1) & 7);
        const int rb2 = kR32Rg * w + 272 * s + 136 * ((tk >> 4) & 1) + kR32Row * ((tk >> 5) & 7);
        const int wb2 = kR32Rg * w + 272 * s + gam;
        double2 R1[16], R2[16];
#pragma unroll
        for (int kl = 0; kl < 8; ++kl) {
            flds[wb2 + kR32Row * kl] = c[kl];
            flds[wb2 + 136 + kR32Row * kl] = c[16 + kl];
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) R1[i] = flds[rb1 + i];
        wave_lds_sync();
#pragma unroll
        for (int kl = 0; kl < 8; ++kl) {
            flds[wb2 + kR32Row * kl] = c[8 + kl];
            flds[wb2 + 136 + kR32Row * kl] = c[24 + kl];
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) R2[i] = flds[rb2 + i];
        Probe::stamp(8, rnd);
        // ---- stage 3: DFT16 over gamma -> lambda
        dft16f(R1);
        dft16f(R2);
        Probe::stamp(9, rnd);
        // ---- pair step: slot i pairs R1[i] (bin k) with R2[15 - i] (bin N - k);
        // the special lane permutes its registers into that layout first
        const bool sp = wu == 0 && lane == kR16SpecialLane;
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
            // the second half's entry 8 + i into the registers pair i has
            // just freed, so each load has the remaining pairs to land in
            pq[8 + i] = pair[j + kR16NT * (8 + i)];
            if (i & 1) p2v[4 + (i >> 1)] = pair[j + kR16NT * (20 + (i >> 1))];
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 8; i < 16; ++i) {
            fft_pair_sym(R1[i], R2[15 - i], pq[i].x, pq[i].y, (i & 1) ? p2v[i >> 1].y : p2v[i >> 1].x, R1[i],
                         R2[15 - i]);
            __builtin_amdgcn_sched_barrier(0);
        }
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
        Probe::stamp(10, rnd);
        // ---- inverse stage 3: DFT16 over lambda -> gamma (on conj(V))
        dft16f(R1);
        dft16f(R2);
        Probe::stamp(11, rnd);
        // ---- T2 backwards (addresses recomputed from laundered words)
        {
            uint32_t tkb = tk_all;
            int jb = threadIdx.x;
            asm volatile("" : "+v"(tkb), "+v"(jb));
            const int wb_ = jb >> 6, sb_ = (jb >> 4) & 3, gmb = jb & 15;
            const int sb1 = kR32Rg * wb_ + 272 * sb_ + 136 * (tkb & 1) + kR32Row * ((tkb >> 1) & 7);
            const int sb2 = kR32Rg * wb_ + 272 * sb_ + 136 * ((tkb >> 4) & 1) + kR32Row * ((tkb >> 5) & 7);
            const int sbw = kR32Rg * wb_ + 272 * sb_ + gmb;
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[sb1 + i] = R1[i];
            wave_lds_sync();
#pragma unroll
            for (int kl = 0; kl < 8; ++kl) {
                c[kl] = flds[sbw + kR32Row * kl];
                c[16 + kl] = flds[sbw + 136 + kR32Row * kl];
            }
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[sb2 + i] = R2[i];
            wave_lds_sync();
#pragma unroll
            for (int kl = 0; kl < 8; ++kl) {
                c[8 + kl] = flds[sbw + kR32Row * kl];
                c[24 + kl] = flds[sbw + 136 + kR32Row * kl];
            }
        }
        Probe::stamp(12, rnd);
        // ---- inverse stage 2: * W_256^(gam kappa), DFT16 over kappa -> beta.
        // The powers are rebuilt, not kept from stage 2 (the laundered base
        // stops the compiler from holding them across the pair step).
        asm volatile("" : "+v"(wg.x), "+v"(wg.y));
        {
            const double2 w2 = cmul(wg, wg);
            const double2 w4 = cmul(w2, w2);
            const double2 one = make_double2(1.0, 0.0);
            r32_chain_anchored<16>(c, 0, one, wg, w4);
            r32_chain_anchored<16>(c, 16, one, wg, w4);
        }
        {
            double2 cA[16], cB[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                cA[i] = c[i];
                cB[i] = c[16 + i];
            }
            dft16f(cA);
            dft16f(cB);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                c[i] = cA[i];
                c[16 + i] = cB[i];
            }
        }
        wave_lds_sync();
        Probe::stamp(13, rnd);
        // ---- T1 backwards, round 1: pair A (column P) into the wave's own
        // region, slot 256 s + thread (16 beta + gam); thread b reads k1 < 16
        // from the region of column k1's reader
        {
            const int base = kR32Rg * w + 256 * s + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[base + 16 * i] = c[i];
        }
        r32_bar();
        Probe::stamp(14, rnd);
        {
            int jr = threadIdx.x;
            asm volatile("" : "+v"(jr));
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int home = r16_home(r); // uniform
                a[r] = flds[kR32Rg * (home >> 2) + 256 * (home & 3) + jr];
            }
        }
        r32_bar();
        Probe::stamp(15, rnd);
        // ---- T1 backwards, round 2: pair B (column r16_col_b(P)) into the
        // region of thread 16 beta + gam, row (column & 15)
        {
            const int base = 64 * (r16_col_b(P) & 15) + gam;
#pragma unroll
            for (int i = 0; i < 16; ++i) flds[base + kR32Rg * (i >> 2) + 16 * (i & 3)] = c[16 + i];
        }
        r32_bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) a[16 + i] = flds[kR32Rg * w + 64 * i + lane];
        Probe::stamp(16, rnd);
        // ---- final: * W_8192^(b k1), DFT32 over k1 -> n
        {
            double2 wb = twl[kR16TwB + j];
            asm volatile("" : "+v"(wb.x), "+v"(wb.y));
            r32_chain32acc(a, wb);
        }
        dft32(a);
        Probe::stamp(17, rnd);
        const float pk = r16_store_unit(p, ch, n0, B, j, a);
        if (ch != pk_ch) {
            if (p.peak && pk_ch >= 0) {
                r16_peak_stage(pk_lds, pk_run);
                pk_pending = pk_ch;
                asm volatile("" : "+v"(pk_pending));
            }
            pk_run = 0.0f;
            pk_ch = ch;
        }
        pk_run = fmaxf(pk_run, pk);
        Probe::stamp(18, rnd);
    }
    if (p.peak && pk_ch >= 0) {
        __syncthreads();
        if (pk_pending >= 0 && threadIdx.x == 0) r16_peak_commit(p, pk_pending, pk_lds);
        __syncthreads();
        r16_peak_stage(pk_lds, pk_run);
        __syncthreads();
        if (threadIdx.x == 0) r16_peak_commit(p, pk_ch, pk_lds);
    }
}

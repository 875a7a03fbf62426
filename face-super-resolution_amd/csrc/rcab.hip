// Fused RCAB forward (reference src/models/blocks.py:135-153 with ChannelAttention
// blocks.py:83-92): one launch computes, per 16x16-pixel tile and all 64 channels,
//
//   z1 = conv1(x) + b1          (on the 18x18 region conv2 needs: halo recompute)
//   a1 = PReLU(z1)              (zero outside the image = conv2's zero padding)
//   t  = conv2(a1) + b2         (16x16)
//   s  = sigmoid(W2 relu(W1 mean_hw(t)))   (per image: needs every tile of the image)
//   y  = t * s * res_scale + x
//
// bf16 activations, fp32 MFMA accumulation, C = 64, Cr <= 16, H and W multiples of 16.
//
// Structure (one 512-thread block per CU, persistent; tiles walked in rounds that cover
// whole images, so every tile an image needs is resident in the same round):
//   * x halo of the tile (20x20 px) + a 4-column edge copy streamed by LDS-DMA, one tile
//     ahead;
//   * the two filters stream tap by tap from L2 through a 6-slot LDS ring (3 taps per
//     phase, refilled one phase ahead) -- both filters (144 KB) do not fit next to the
//     activation images;
//   * conv1 (21 pixel fragments: 18 rows of 16 + 3 fragments of the 2 edge columns) ->
//     bias + PReLU -> a1 image in LDS; conv2 reads it with the halo-row-reuse MFMA order;
//   * t stays in registers.  The tile's pool partial goes to an uncached workspace, then
//     the block arrives on its image's counter (MI355X_MICROARCH.md 'inter-workgroup
//     visibility': the per-XCD L2s are not coherent, so the hand-off bypasses them).
//     One phase boundary into its NEXT tile, wave 0 polls the counter, sums the image's
//     partials in a fixed order (deterministic), computes the gate (FC-ReLU-FC-sigmoid)
//     into LDS, and after the next barrier every wave applies y = t*s*rs + x; the last
//     tile does the same right away.  The counters clean themselves up (the last reader
//     of an image resets them), so a hipGraph can replay the launch.
#include "fen_common.h"

namespace {

constexpr int XW = 20;                       // conv1 input halo, 20x20 px
constexpr int XH_BYTES = XW * XW * 128;      // 51200 = 50 DMA pieces
constexpr int XH_DMA = XH_BYTES / 1024;
constexpr int EH_BYTES = XW * 4 * 128;       // halo columns 16..19 again, row-keyed: 10 pieces
constexpr int EH_DMA = EH_BYTES / 1024;
constexpr int HALO_W = (XH_DMA + EH_DMA) / 8;   // halo pieces per wave (+1 for the first waves)
constexpr int A1W = 18;                      // a1 image = conv2 halo, 18x18, hcol layout
constexpr int A1_BYTES = A1W * A1W * 128;    // 41472
constexpr int TAP_BYTES = 64 * 128;          // one filter tap [64 co][64 ci] bf16
constexpr int O_XH = 0;
constexpr int O_EH = O_XH + XH_BYTES;
constexpr int O_A1 = O_EH + EH_BYTES;
constexpr int O_RING = O_A1 + A1_BYTES;
constexpr int O_RED = O_RING + 6 * TAP_BYTES;   // [4][64] f32 pool partials of the 4 row waves
constexpr int O_CST = O_RED + 4 * 64 * 4;       // b1[64] alpha[64] b2[64]
constexpr int O_FC = O_CST + 3 * 64 * 4;        // fc1 [16][64], fc2 [64][16] f32
constexpr int O_FLAG = O_FC + 2 * 1024 * 4;     // block-wide scalars
#ifdef FEN_STAMPS
constexpr int O_STAMP = O_FLAG + 64;            // diagnostic build: [8 waves][48] u32 stamps
constexpr int RCAB_LDS = O_STAMP + 8 * 48 * 4;
#else
constexpr int RCAB_LDS = O_FLAG + 64;
#endif
static_assert(RCAB_LDS <= 163840, "LDS budget");
static_assert(O_RING % 16 == 0 && O_RED % 16 == 0 && O_FC % 16 == 0, "alignment");

// diagnostic build (-DFEN_STAMPS): s_memrealtime per wave at phase points into d.stamps,
// [block][wave][48]; the product build executes none of it
// The stamps land in LDS (low 32 bits; copied out once at the end of the kernel): a global
// store per stamp would sit in vmcnt and stretch every boundary's vmcnt(0) wait.
#ifdef FEN_STAMPS
#define RSTAMP(i)                                                                            \
    do {                                                                                     \
        unsigned long long _rt;                                                              \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_rt)::"memory");      \
        if (lane == 0 && (i) < 48) stamp_lds[wave * 48 + (i)] = (unsigned)_rt;                 \
    } while (0)
#else
#define RSTAMP(i) \
    do {          \
    } while (0)
#endif

constexpr int MAX_GRID = 1024;               // start-flag slots (grid <= CUs)
constexpr int CP_SC = 17;                     // buffer cache policy sc0|sc1: straight to memory
constexpr unsigned POLL_MAX = 1u << 20;      // ~0.5 s of s_sleep: a gate that never comes
                                             // sets sync[3*B] and the kernel exits anyway

// 16-B chunk position in the edge image: pixel e = row*4 + col', key = (2 row) & 7.  Checked
// against ds_read_b128's lane groups for every (edge fragment, kh, kw, k-half): conflict-free;
// the key row & 7 left 2-way conflicts in a third of them (tools note in DESIGN.md)
__device__ __forceinline__ int ekey_of(int row) { return (2 * row) & 7; }
__device__ __forceinline__ int ekey(int row, int chunk) { return (chunk ^ ekey_of(row)) << 4; }

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Output stores nobody in this launch reads again (y; training copies of z1 / a1).  Plain
// stores: the non-temporal form (RCAB_NT, meant to keep x in L2 for the apply one tile
// later) measured neutral for inference (42.3 us both) and 1.45x SLOWER for training
// (74.7 vs 51.2 us: the 8-B fragment-layout pieces then reach HBM as partial-line writes
// instead of merging in L2) -- tools/gpu_ab_rcab.sh
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_out16(void* p, uint4 v) {
#ifndef RCAB_NT
    *(uint4*)p = v;
#else
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4*)p);
#endif
}
template <typename T>
__device__ __forceinline__ void st_out4(void* p, const float v[4]) {
    const unsigned lo = (unsigned)to16<T>(v[0]) | ((unsigned)to16<T>(v[1]) << 16);
    const unsigned hi = (unsigned)to16<T>(v[2]) | ((unsigned)to16<T>(v[3]) << 16);
#ifndef RCAB_NT
    *(uint2*)p = make_uint2(lo, hi);
#else
    __builtin_nontemporal_store((unsigned long long)lo | ((unsigned long long)hi << 32), (unsigned long long*)p);
#endif
}

// sync-word access (uncached workspace: every load / store goes to memory)
__device__ __forceinline__ int ld_poll(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// conv2 MFMAs for one phase (kernel column kw: taps (0,kw),(1,kw),(2,kw) in ring slots),
// halo-row-reuse order on the a1 image; wave = 4 output rows x 32 channels.
template <typename T>
__device__ __forceinline__ void conv2_phase(f32x4 (&acc)[2][4], const char* a1, const char* const (&tapp)[3], int kw,
                                            int wr, int arow, int q, int c16) {
    uint4 A0[3][2], B0[6], A1[3][2], B1[6];
    auto load = [&](int kk, uint4 (&A)[3][2], uint4 (&Bf)[6]) {
        const int chunk = kk * 4 + q;
        const char* hb = a1 + hcol(c16 + kw, chunk) + (wr * 4) * (A1W * 128);
#pragma unroll
        for (int n = 0; n < 6; ++n) Bf[n] = *(const uint4*)(hb + n * (A1W * 128));
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int m = 0; m < 2; ++m) A[kh][m] = *(const uint4*)(tapp[kh] + swz(arow + m * 16, chunk));
    };
    auto mma = [&](const uint4 (&A)[3][2], const uint4 (&Bf)[6]) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) mma16<T>(acc[m][n], A[kh][m], Bf[n + kh]);
    };
    load(0, A0, B0);
    load(1, A1, B1);
    __builtin_amdgcn_sched_barrier(0);
    mma(A0, B0);
    __builtin_amdgcn_sched_barrier(0);
    mma(A1, B1);
    __builtin_amdgcn_sched_barrier(0);
}

// conv1 for one phase = kernel column kw (taps (0,kw),(1,kw),(2,kw) in ring slots 0..2), the
// halo-row-reuse order conv2 uses: per k-half the wave loads its NR + 2 input rows once and
// reuses them across the 3 kernel rows (13-18 fragment reads for 30-36 MFMAs; the by-row
// order read 0.67-0.7 fragments per MFMA in 6 interleaved steps).  Slots 0..NR-1 are main
// rows row0.. (16 columns); without MAIN4 slot 4 is edge fragment eidx4, with HAS5 slot 5 is
// edge fragment 1 (edge reads do not reuse across kh: their lanes map to (row, column)).
__device__ __forceinline__ int edge_base(int eidx, int c16, int kh, int chunk) {
    int r = 8 * eidx + (c16 >> 1);
    if (r > 17) r = 17;
    return ((r + kh) * 4 + (c16 & 1)) * 128 + ekey(r + kh, chunk);
}
template <typename T, bool MAIN4, bool HAS5>
__device__ __forceinline__ void conv1_kw(f32x4 (&acc)[2][6], const char* xh, const char* eh,
                                         const char* const (&tapp)[3], int kw, int c16, int row0, int eidx4,
                                         int arow, int q) {
    constexpr int NR = MAIN4 ? 5 : 4;
    constexpr int NB = NR + 2;
    // opaque lane coordinates: every address below is recomputed per phase instead of being
    // hoisted out of the tile loop (12 loop-invariant edge / A offsets live through conv2,
    // the kernel's register peak, spilled)
    asm volatile("" : "+v"(c16), "+v"(arow), "+v"(q));
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + q;
        const char* xb = xh + hcol(c16 + kw, chunk) + row0 * (XW * 128);
        uint4 Bm[NB], A[3][2], E4[3], E5[3];
#pragma unroll
        for (int j = 0; j < NB; ++j) Bm[j] = *(const uint4*)(xb + j * (XW * 128));
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int m = 0; m < 2; ++m) A[kh][m] = *(const uint4*)(tapp[kh] + swz(arow + m * 16, chunk));
        if constexpr (!MAIN4) {
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) E4[kh] = *(const uint4*)(eh + edge_base(eidx4, c16, kh, chunk) + kw * 128);
        }
        if constexpr (HAS5) {
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) E5[kh] = *(const uint4*)(eh + edge_base(1, c16, kh, chunk) + kw * 128);
        }
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int m = 0; m < 2; ++m) {
#pragma unroll
                for (int f = 0; f < NR; ++f) mma16<T>(acc[m][f], A[kh][m], Bm[f + kh]);
                if constexpr (!MAIN4) mma16<T>(acc[m][4], A[kh][m], E4[kh]);
                if constexpr (HAS5) mma16<T>(acc[m][5], A[kh][m], E5[kh]);
            }
#ifdef RCAB_C1_FENCE
        __builtin_amdgcn_sched_barrier(0);   // A/B only: one k-half's fragments live at a time
#endif
    }
}

// ------------------------------------------------------------------------------------
// the kernel
// ------------------------------------------------------------------------------------
// PARK (training, d.t given): t is parked in d.t (stored for the backward anyway) and the
// apply re-reads it with coalesced 16-B loads; else t stays in 16 VGPRs (packed bf16) and the
// apply uses the MFMA fragment layout (fewer HBM bytes, more registers).
template <typename T, bool PARK>
__global__ __launch_bounds__(512, 1) void k_rcab(const fen_rcab_desc d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* xh = smem + O_XH;
    char* eh = smem + O_EH;
    char* a1s = smem + O_A1;
    char* ring = smem + O_RING;
    float* red = (float*)(smem + O_RED);
    float* cst = (float*)(smem + O_CST);
    float* fcs = (float*)(smem + O_FC);
    int* lflag = (int*)(smem + O_FLAG);
#ifdef FEN_STAMPS
    unsigned* stamp_lds = (unsigned*)(smem + O_STAMP);
    for (int i = threadIdx.x; i < 8 * 48; i += blockDim.x) stamp_lds[i] = 0u;
    __syncthreads();
#endif

    const int tid = threadIdx.x, lane = tid & 63;
    // the wave id through readfirstlane: provably wave-uniform to the compiler, so the
    // per-wave roles (conv1 fragment group: slot-4 main/edge, slot 5; wave 0's gate; the
    // opt-in s_setprio of waves 4-7) compile to scalar branches.  tid >> 6 alone is divergent to
    // hipcc: the slot-5 MFMAs and reads were exec-masked (issued by every wave) and
    // s_setprio 1 ran unconditionally in all waves (cdna_hip_programming.md, s_setprio
    // recipe / descriptor recipe).  RCAB_DIV_WAVE: the old form, for A/B.
#ifdef RCAB_DIV_WAVE
    const int wave = tid >> 6;
#else
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#endif
    const int q = lane >> 4, c16 = lane & 15;
    const int ch = wave & 1, g = wave >> 1;          // conv1: channel half, fragment group
    const int wr = wave >> 1, wc = wave & 1;         // conv2: row group, channel half
    const int H = d.H, W = d.W, B = d.B, Cr = d.Cr;
    const int twn = W >> 4, tpi = twn * (H >> 4);
    const int ntiles = B * tpi;
    const int nslot = gridDim.x;
    // XCD-aware slot: blocks b and b + 8 share an XCD (round-robin dispatch, observed), so
    // slot = (b % 8) * (nslot / 8) + b / 8 puts an image's tiles -- consecutive slots -- on
    // one XCD: neighbouring tiles' halo rows and the apply's re-read of x come from that
    // XCD's L2 instead of another die's copy.  Any permutation is correct (all blocks are
    // co-resident); the mapping only moves traffic.
#ifndef RCAB_NO_XCD
    const int slot = xcd_block();
#else
    const int slot = (int)blockIdx.x;
#endif
    const int nmine = (ntiles - slot + nslot - 1) / nslot;
    // workspace (fen_rcab_workspace_alloc: uncached, so every access of the cross-block
    // hand-off goes to memory -- the per-XCD L2s are not coherent):
    //   part  [tpi][B][64]  tile partial sums, image-interleaved so that one image's rows
    //                       lie B*256 B apart (spread over many HBM channels, not one hot 16 KB)
    //   tflag [tpi][B]      tile arrival flags (= launch epoch + 1 once the partial landed)
    //   sflag [MAX_GRID]    block start flags (= epoch + 1 once the block has read the epoch)
    //   epoch, err
    // No atomics and no resets: flags only ever move to the current epoch + 1, and block 0
    // advances the epoch at its end, once every block of the launch has read it.
    float* part = (float*)d.ws;
    int* tflag = (int*)(part + (size_t)ntiles * 64);
    int* sflag = tflag + ntiles;
    int* epoch = sflag + MAX_GRID;
    int* err = epoch + 1;
    const __amdgpu_buffer_rsrc_t partr =
        __builtin_amdgcn_make_buffer_rsrc(part, 0, (int)((size_t)ntiles * 256), 0x00020000);

    const i32x4 xr4 = make_rsrc(d.x, (unsigned)((size_t)B * H * W * 128));
    const i32x4 w1r = make_rsrc(d.w1, 9u * 64u * 128u);
    const i32x4 w2r = make_rsrc(d.w2, 9u * 64u * 128u);

    // ring: phase P of the block's sequence (6 per tile) uses slots (P & 1) * 3 + i.
    // phase p = 0..2: conv1 taps 3p..3p+2; p = 3..5: conv2 taps (kh, kw = p - 3), kh = 0..2
    auto issue_taps = [&](int P) {
        const int p = P % 6;
        char* base = ring + (P & 1) * 3 * TAP_BYTES;
        const int s = wave * 64 + lane, r = s >> 3, pc = s & 7;
        const int c = pc ^ ((r >> 1) & 7);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int tap = i * 3 + (p < 3 ? p : p - 3);   // slot i = tap (kh = i, kw = phase)
            const int voff = ((tap * 64 + r) * 64 + c * 8) * 2;
            dma16(p < 3 ? w1r : w2r, __builtin_amdgcn_readfirstlane(lds_addr(base + i * TAP_BYTES + wave * 1024)),
                  voff);
        }
    };
    // x halo (20x20, hcol key) + edge copy (halo columns 16..19, row key) of tile t
    auto issue_halo = [&](int t) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        for (int i = wave; i < XH_DMA + EH_DMA; i += 8) {
            int voff = 0x7ffffff0;
            unsigned base;
            if (i < XH_DMA) {
                const int s = i * 64 + lane, p = s >> 3, pc = s & 7;
                const int hr = p / XW, hc = p - hr * XW;
                const int c = pc ^ (hc & 7);
                const int gh = h0 - 2 + hr, gw = w0 - 2 + hc;
                if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W) voff = (((b * H + gh) * W + gw) * 64 + c * 8) * 2;
                base = lds_addr(xh + i * 1024);
            } else {
                const int s = (i - XH_DMA) * 64 + lane, e = s >> 3, pc = s & 7;
                const int hr = e >> 2, hc = 16 + (e & 3);
                const int c = pc ^ ekey_of(hr);
                const int gh = h0 - 2 + hr, gw = w0 - 2 + hc;
                if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W) voff = (((b * H + gh) * W + gw) * 64 + c * 8) * 2;
                base = lds_addr(eh + (i - XH_DMA) * 1024);
            }
            dma16(xr4, __builtin_amdgcn_readfirstlane(base), voff);
        }
    };

    // ---- start-up: first taps + first halo (LDS-DMA) go out before anything waits on memory;
    //      then constants, SE weights and the epoch read, whose round trips overlap the DMA
#ifndef RCAB_OLD_PROLOGUE
    issue_taps(0);
    issue_halo(slot);
#endif
    if (tid < 64) {
        cst[tid] = d.b1[tid];
        cst[64 + tid] = d.alpha[tid];
        cst[128 + tid] = d.b2[tid];
    }
    for (int i = tid; i < 1024; i += 512) {           // both zero-padded to 16 hidden units
        fcs[i] = i < Cr * 64 ? d.fc1[i] : 0.f;          // [16][64]
        const int c = i >> 4, j = i & 15;
        fcs[1024 + i] = j < Cr ? d.fc2[c * Cr + j] : 0.f;   // [64][16]
    }
#ifdef RCAB_PRIO
    // waves 4-7 at priority 1 (MI355X_MICROARCH.md 'Two waves per SIMD'): measured ~1 us
    // SLOWER per launch once the wave id is uniform (before that, s_setprio ran in every
    // wave, a no-op) -- opt-in for A/B only
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    // this launch's epoch; announce that this block has read it
    const int ep1 = __builtin_amdgcn_readfirstlane(ld_poll(epoch)) + 1;
    if (tid == 0) st_flag(sflag + blockIdx.x, ep1);
    RSTAMP(0);
#ifdef RCAB_OLD_PROLOGUE
    issue_taps(0);
    issue_halo(slot);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    RSTAMP(1);

    // conv1 per-lane addressing (group g: rows row0.., slot 4 main for g < 2, edges for g >= 2)
    const int row0 = g == 0 ? 0 : g == 1 ? 5 : g == 2 ? 10 : 14;
    const bool main4 = g < 2, has5 = g == 3;
    const int eidx4 = g == 2 ? 2 : 0;
    const int arow1 = ch * 32 + c16;                  // A row (co) of conv1's wave
    const int arow2 = wc * 32 + c16;
    // conv1 epilogue addressing, fixed per lane: a1-image byte offsets of slot 0 (main rows:
    // + f * 2304) and of slots 4, 5 (main row 4 or an edge fragment; edge pad lanes write a
    // dummy word), and each slot's (row, column) in a1 coordinates
    const int ar4 = main4 ? row0 + 4 : 8 * (g == 2 ? 2 : 0) + (c16 >> 1), ac4 = main4 ? c16 : 16 + (c16 & 1);
    const int ar5 = 8 + (c16 >> 1), ac5 = 16 + (c16 & 1);
    int a1m[2], a1o4[2], a1o5[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int chunk = ch * 4 + 2 * m + (q >> 1);
        a1m[m] = (row0 * A1W + c16) * 128 + ((chunk ^ (c16 & 7)) << 4) + (q & 1) * 8;
        a1o4[m] = ar4 <= 17 ? (ar4 * A1W + ac4) * 128 + ((chunk ^ (ac4 & 7)) << 4) + (q & 1) * 8 : O_FLAG - O_A1;
        a1o5[m] = (ar5 * A1W + ac5) * 128 + ((chunk ^ (ac5 & 7)) << 4) + (q & 1) * 8;
    }

    // t (bf16) of the tile awaiting its gate: parked in d.t (PARK) or carried in tcar
    T* const tpark = (T*)d.t;
    uint2 tcar[2][4];
    (void)tcar;
    int arrive_f = -1;                                // tile flag still to be raised
    auto arrive = [&]() {                             // after an s_waitcnt vmcnt(0) of wave 0
        if (arrive_f >= 0 && tid == 0) st_flag(tflag + arrive_f, ep1);
        arrive_f = -1;
    };
    int pend_t = -1;                                  // that tile (-1: none)

    // The SE gate of image b, by wave 0 alone, into LDS (gsh[0..63] = s, read by every wave
    // after the next barrier).  Poll the arrival counter, read the image's tpi partials with
    // 16-B uncached loads (4 rows per instruction), fixed-order sums, mean -> FC1 -> ReLU ->
    // FC2 -> sigmoid; `first` tiles write the user copies.
    float* gsh = red;                                 // s of the pending tile (red is free then)
    auto gate_to_lds = [&](int b, bool first, int sb) {
        {   // every tile of the image has raised its flag (lane i watches tiles i, i+64, ..)
            unsigned it = 0;
            for (;;) {
                bool mine = true;
                for (int i = lane; i < tpi; i += 64) mine &= ld_poll(tflag + i * B + b) == ep1;
                if (__all(mine) || ++it >= POLL_MAX) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (it >= POLL_MAX && lane == 0) st_flag(err, 1);
        }
        RSTAMP(sb);
        const int rg = lane >> 4, c4 = (lane & 15) * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        asm volatile("" ::: "memory");                // the loads stay behind the poll
        for (int r0 = 0; r0 < tpi; r0 += 16) {
            unsigned __attribute__((ext_vector_type(4))) v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = min(r0 + 4 * j + rg, tpi - 1);
                v[j] = __builtin_amdgcn_raw_buffer_load_b128(partr, ((r * B + b) * 64 + c4) * 4, 0, CP_SC);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (r0 + 4 * j + rg < tpi) {
                    acc.x += __uint_as_float(v[j][0]); acc.y += __uint_as_float(v[j][1]);
                    acc.z += __uint_as_float(v[j][2]); acc.w += __uint_as_float(v[j][3]);
                }
            }
        }
        RSTAMP(sb + 1);
        // fold the 4 row groups through LDS (red[4][64] -> mean in red[0..63]), then
        // FC1: lane = (part, j) dots 16 channels of mean with fc1 row j, two xor folds;
        // FC2: lane c dots the 16 (zero-padded) hidden units with fc2 row c.  A handful of
        // dependent LDS round trips instead of a wave reduction per hidden unit.
        *(float4*)(red + rg * 64 + c4) = acc;
        const float mean = ((red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane])) * d.inv_hw;
        red[lane] = mean;
        const int j = lane & 15, part4 = lane >> 4;
        float h = 0.f;
#pragma unroll
        for (int c = 0; c < 16; c += 4) {
            const float4 w = *(const float4*)(fcs + j * 64 + part4 * 16 + c);
            const float4 m = *(const float4*)(red + part4 * 16 + c);
            h += w.x * m.x + w.y * m.y + w.z * m.z + w.w * m.w;
        }
        h += __shfl_xor(h, 16, 64);
        h += __shfl_xor(h, 32, 64);
        const float hid_mine = fmaxf(h, 0.f);         // hidden unit j (0 for j >= Cr)
        if (lane < 16) red[64 + lane] = hid_mine;
        float z = 0.f;
#pragma unroll
        for (int c = 0; c < 16; c += 4) {
            const float4 w = *(const float4*)(fcs + 1024 + lane * 16 + c);
            const float4 hv = *(const float4*)(red + 64 + c);
            z += w.x * hv.x + w.y * hv.y + w.z * hv.z + w.w * hv.w;
        }
        const float sg = 1.f / (1.f + expf(-z));
        gsh[lane] = sg;
        RSTAMP(sb + 2);
        if (first) {                                  // the user-visible copies, once per image
            d.s[(size_t)b * 64 + lane] = sg;
            if (d.mean) d.mean[(size_t)b * 64 + lane] = mean;
            if (d.hid && lane < Cr) d.hid[(size_t)b * Cr + lane] = hid_mine;
        }
    };

    // y = t * s * rs + x for tile `pt` (t parked, s in gsh), coalesced: wave w owns tile
    // rows 2w, 2w+1 (4 KB); lane l moves 16-B chunks i*64 + l (8 full 128-B pixel rows
    // per instruction) -- a quarter of the requests of the MFMA-fragment layout
    uint4 xv[4], tv[4];   // PARK
    auto load_x = [&](int pt) {
        const int b = pt / tpi, tile = pt - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = i * 64 + lane, p = g >> 3, c = g & 7;
            const size_t o = ((size_t)(b * H + h0 + wave * 2 + (p >> 4)) * W + w0 + (p & 15)) * 128 + c * 16;
            xv[i] = *(const uint4*)((const char*)d.x + o);
            tv[i] = *(const uint4*)((const char*)tpark + o);
        }
    };
    auto apply = [&](int pt) {                        // after load_x(pt)
        const int b = pt / tpi, tile = pt - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const float rs = d.res_scale;
        const int c = lane & 7;                       // the same chunk in every iteration
        const float4 s0 = *(const float4*)(gsh + c * 8), s1 = *(const float4*)(gsh + c * 8 + 4);
        const float sv[8] = {s0.x * rs, s0.y * rs, s0.z * rs, s0.w * rs, s1.x * rs, s1.y * rs, s1.z * rs, s1.w * rs};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = i * 64 + lane, p = g >> 3;
            const size_t o = ((size_t)(b * H + h0 + wave * 2 + (p >> 4)) * W + w0 + (p & 15)) * 128 + c * 16;
            const unsigned tw[4] = {tv[i].x, tv[i].y, tv[i].z, tv[i].w}, xw[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
            unsigned ow[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float lo = lo16<T>(tw[e]) * sv[2 * e] + lo16<T>(xw[e]);
                const float hi = hi16<T>(tw[e]) * sv[2 * e + 1] + hi16<T>(xw[e]);
                ow[e] = (unsigned)to16<T>(lo) | ((unsigned)to16<T>(hi) << 16);
            }
            st_out16((char*)d.y + o, make_uint4(ow[0], ow[1], ow[2], ow[3]));
        }
    };
    // (!PARK) y = t * s * rs + x in the MFMA fragment layout (t in tcar)
    uint2 xf[2][4];
#ifndef RCAB_XLOAD_NOSHFL
    // x as 16-B loads in the paired-lane layout of the y stores (even lane q: m = 0 channels
    // 4q..4q+7, odd: m = 1 channels 4(q-1)..4q+3); apply_frag trades the halves back
    uint4 xr[4];
    auto load_x_frag = [&](int pt) {
        const int b = pt / tpi, tile = pt - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const size_t px = (size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16;
            xr[n] = *(const uint4*)((const char*)d.x + (px * 64 + wc * 32 + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q)) * 2);
        }
    };
    auto unpair_x = [&]() {
        const bool odd = q & 1;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const uint2 lo = make_uint2(xr[n].x, xr[n].y), hi = make_uint2(xr[n].z, xr[n].w);
            const uint2 snd = odd ? lo : hi;
            uint2 rcv;
            rcv.x = (unsigned)__shfl_xor((int)snd.x, 16, 64);
            rcv.y = (unsigned)__shfl_xor((int)snd.y, 16, 64);
            xf[0][n] = odd ? rcv : lo;
            xf[1][n] = odd ? hi : rcv;
        }
    };
#else
    auto load_x_frag = [&](int pt) {
        const int b = pt / tpi, tile = pt - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const size_t px = (size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16;
#pragma unroll
            for (int m = 0; m < 2; ++m) xf[m][n] = *(const uint2*)((const char*)d.x + (px * 64 + wc * 32 + m * 16 + 4 * q) * 2);
        }
    };
    auto unpair_x = [&]() {};
#endif
    auto apply_frag = [&](int pt) {
        const int b = pt / tpi, tile = pt - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const float rs = d.res_scale;
        unpair_x();
        float sv[2][4];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float4 s4 = *(const float4*)(gsh + wc * 32 + m * 16 + 4 * q);
            sv[m][0] = s4.x * rs; sv[m][1] = s4.y * rs; sv[m][2] = s4.z * rs; sv[m][3] = s4.w * rs;
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const size_t px = (size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16;
#ifndef RCAB_APPLY_NOSHFL
            // lanes q and q ^ 1 (16 lanes apart) trade one 4-channel half: the even lane stores
            // m = 0 channels 4q..4q+7, the odd lane m = 1 channels 4(q-1)..4q+3, as 16-B stores
            // (64 contiguous bytes per pixel per instruction instead of 32)
            uint2 pk[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                float o[4];
                o[0] = lo16<T>(tcar[m][n].x) * sv[m][0] + lo16<T>(xf[m][n].x);
                o[1] = hi16<T>(tcar[m][n].x) * sv[m][1] + hi16<T>(xf[m][n].x);
                o[2] = lo16<T>(tcar[m][n].y) * sv[m][2] + lo16<T>(xf[m][n].y);
                o[3] = hi16<T>(tcar[m][n].y) * sv[m][3] + hi16<T>(xf[m][n].y);
                pk[m].x = (unsigned)to16<T>(o[0]) | ((unsigned)to16<T>(o[1]) << 16);
                pk[m].y = (unsigned)to16<T>(o[2]) | ((unsigned)to16<T>(o[3]) << 16);
            }
            const bool odd = q & 1;
            const uint2 snd = odd ? pk[0] : pk[1];
            uint2 rcv;
            rcv.x = (unsigned)__shfl_xor((int)snd.x, 16, 64);
            rcv.y = (unsigned)__shfl_xor((int)snd.y, 16, 64);
            const uint4 v = odd ? make_uint4(rcv.x, rcv.y, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, rcv.x, rcv.y);
            st_out16((char*)d.y + (px * 64 + wc * 32 + (odd ? 16 + 4 * (q - 1) : 4 * q)) * 2, v);
#else
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                float o[4];
                o[0] = lo16<T>(tcar[m][n].x) * sv[m][0] + lo16<T>(xf[m][n].x);
                o[1] = hi16<T>(tcar[m][n].x) * sv[m][1] + hi16<T>(xf[m][n].x);
                o[2] = lo16<T>(tcar[m][n].y) * sv[m][2] + lo16<T>(xf[m][n].y);
                o[3] = hi16<T>(tcar[m][n].y) * sv[m][3] + hi16<T>(xf[m][n].y);
                st_out4<T>((char*)d.y + (px * 64 + wc * 32 + m * 16 + 4 * q) * 2, o);
            }
#endif
        }
    };

#pragma unroll 1
    for (int k = 0; k < nmine; ++k) {
        const int t = slot + k * nslot;
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        f32x4 acc1[2][6];
        // ================= conv1: phases 0..2 =================
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int f = 0; f < 6; ++f) acc1[m][f] = zero4();
#pragma unroll 1
        for (int p = 0; p < 3; ++p) {
            const int P = k * 6 + p;
            if (p > 0 || k > 0) {
                if (k < 2) RSTAMP(2 + k * 14 + p * 2);
                if (p == 0 && wave == 0) {
                    // the last tile's partial store (this wave's newest op) keeps draining to
                    // memory through phase 0; its arrival is raised at the next boundary
                    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this phase's taps (+ halo) landed
                    arrive();                                          // ... and the last tile's partial
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (k < 2) RSTAMP(3 + k * 14 + p * 2);
            }
            issue_taps(P + 1);
            const char* tapp[3] = {ring + (P & 1) * 3 * TAP_BYTES, ring + (P & 1) * 3 * TAP_BYTES + TAP_BYTES,
                                   ring + (P & 1) * 3 * TAP_BYTES + 2 * TAP_BYTES};
            if (k == 1 && p == 1) RSTAMP(45);
            if (g < 2) conv1_kw<T, true, false>(acc1, xh, eh, tapp, p, c16, row0, eidx4, arow1, q);
            else if (g == 2) conv1_kw<T, false, false>(acc1, xh, eh, tapp, p, c16, row0, eidx4, arow1, q);
            else conv1_kw<T, false, true>(acc1, xh, eh, tapp, p, c16, row0, eidx4, arow1, q);
            if (k == 1 && p == 1) RSTAMP(46);
        }
        if (k == 0) RSTAMP(15);
        // ---- conv1 epilogue: bias + PReLU -> a1 image (zero outside the image; branch-free,
        //      precomputed offsets); training copies of z1 / a1 for the backward (16x16 interior)
        {
            const bool colok = (unsigned)(w0 - 1 + c16) < (unsigned)W;
            const bool ok4 = (unsigned)(h0 - 1 + ar4) < (unsigned)H && (unsigned)(w0 - 1 + ac4) < (unsigned)W;
            const bool ok5 = (unsigned)(h0 - 1 + ar5) < (unsigned)H && (unsigned)(w0 - 1 + ac5) < (unsigned)W;
            float zs[2][6][4];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const float4 bb = *(const float4*)(cst + ch * 32 + m * 16 + 4 * q);
                const float4 aa = *(const float4*)(cst + 64 + ch * 32 + m * 16 + 4 * q);
                const float bia[4] = {bb.x, bb.y, bb.z, bb.w}, alp[4] = {aa.x, aa.y, aa.z, aa.w};
#pragma unroll
                for (int f = 0; f < 6; ++f) {
                    bool ok;
                    if (f < 4) ok = colok && (unsigned)(h0 - 1 + row0 + f) < (unsigned)H;
                    else ok = f == 4 ? ok4 : ok5;
                    const float okf = ok ? 1.f : 0.f;
                    float a[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float z = acc1[m][f][r] + bia[r];
                        zs[m][f][r] = z;
                        a[r] = okf * prelu_f(z, alp[r]);
                    }
                    const int off = f < 4 ? a1m[m] + f * (A1W * 128) : f == 4 ? a1o4[m] : a1o5[m];
                    if (f < 5 || has5) st4<T>(a1s + off, a);
                }
            }
#if !defined(RCAB_Z1_LDS) && !defined(RCAB_A1_MASKED) && !defined(RCAB_Z1_NOSHFL)
            if (d.z1) {
                // interior pixels only (a1 rows / cols 1..16), training only: lanes q and q^1
                // (same pixel) trade one 4-channel half so each store is 16 B (see apply_frag)
                const bool odd = q & 1;
#pragma unroll
                for (int f = 0; f < 6; ++f) {
                    uint2 pk[2];
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        pk[m].x = (unsigned)to16<T>(zs[m][f][0]) | ((unsigned)to16<T>(zs[m][f][1]) << 16);
                        pk[m].y = (unsigned)to16<T>(zs[m][f][2]) | ((unsigned)to16<T>(zs[m][f][3]) << 16);
                    }
                    const uint2 snd = odd ? pk[0] : pk[1];
                    uint2 rcv;
                    rcv.x = (unsigned)__shfl_xor((int)snd.x, 16, 64);
                    rcv.y = (unsigned)__shfl_xor((int)snd.y, 16, 64);
                    const int ar = f < 4 ? row0 + f : f == 4 ? ar4 : ar5;
                    const int ac = f < 4 ? c16 : f == 4 ? ac4 : ac5;
                    if (!(f < 5 || has5) || ar < 1 || ar > 16 || ac < 1 || ac > 16) continue;
                    const uint4 v = odd ? make_uint4(rcv.x, rcv.y, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, rcv.x, rcv.y);
                    const size_t o = ((size_t)(b * H + h0 - 1 + ar) * W + w0 - 1 + ac) * 64 + ch * 32 + (odd ? 16 + 4 * (q - 1) : 4 * q);
                    *(uint4*)((char*)d.z1 + o * 2) = v;
                }
            }
#else
            if (d.z1) {
                // interior pixels only (a1 rows / cols 1..16); exec-masked stores, training only
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const float4 aa = *(const float4*)(cst + 64 + ch * 32 + m * 16 + 4 * q);
                    const float alp[4] = {aa.x, aa.y, aa.z, aa.w};
#pragma unroll
                    for (int f = 0; f < 6; ++f) {
                        const int ar = f < 4 ? row0 + f : f == 4 ? ar4 : ar5;
                        const int ac = f < 4 ? c16 : f == 4 ? ac4 : ac5;
                        if (!(f < 5 || has5) || ar < 1 || ar > 16 || ac < 1 || ac > 16) continue;
                        const size_t o = ((size_t)(b * H + h0 - 1 + ar) * W + w0 - 1 + ac) * 64 + ch * 32 + m * 16 + 4 * q;
                        float a[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) a[r] = prelu_f(zs[m][f][r], alp[r]);
#ifndef RCAB_Z1_LDS
                        st_out4<T>((char*)d.z1 + o * 2, zs[m][f]);
#else
                        (void)o;
#endif
#ifdef RCAB_A1_MASKED
                        st_out4<T>((char*)d.a1 + o * 2, a);
#endif
                    }
                }
#ifdef RCAB_Z1_LDS
                // (opt-in, RCAB_Z1_LDS: measured neutral -- the extra barrier costs what the
                // coalesced copy saves) z1 interior -> the x-halo buffer (free once every wave is
                // past conv1: one extra barrier), [16x16 px][8 chunks] with the column-keyed chunk
                // swizzle; copied out as whole pixel rows after the phase-3 barrier
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int f = 0; f < 6; ++f) {
                        const int ar = f < 4 ? row0 + f : f == 4 ? ar4 : ar5;
                        const int ac = f < 4 ? c16 : f == 4 ? ac4 : ac5;
                        if (!(f < 5 || has5) || ar < 1 || ar > 16 || ac < 1 || ac > 16) continue;
                        const int zc = ac - 1, chunk = ch * 4 + 2 * m + (q >> 1);
                        st4<T>(xh + ((ar - 1) * 16 + zc) * 128 + ((chunk ^ (zc & 7)) << 4) + (q & 1) * 8, zs[m][f]);
                    }
#endif
            }
#endif
        }
        // the pending tile's gate (its round ended a conv1 ago): wave 0 -> LDS (RCAB_XPRE:
        // its residual loads go out first, in flight during the gate; costs registers)
#ifdef RCAB_XPRE
        if (pend_t >= 0) {
            if constexpr (PARK) load_x(pend_t);
            else load_x_frag(pend_t);
        }
#endif
        if (pend_t >= 0 && wave == 0) gate_to_lds(pend_t / tpi, pend_t % tpi == 0, 32);
        if (k < 2) RSTAMP(8 + k * 14);
        // ---- phase-3 boundary: a1 image + gate published; apply the pending tile before the
        //      conv2 accumulators come alive (keeps the register peak at the MFMA loops)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (k < 2) RSTAMP(9 + k * 14);
        // vmcnt counts in issue order: the apply (its loads drained by the barrier above) runs
        // before this phase's DMA, and phase 4 waits for its taps only (vmcnt = this wave's
        // halo pieces), leaving the halo in flight until phase 5
#ifdef RCAB_XPRE
        if (pend_t >= 0) {                          // residual landed before the barrier
            if constexpr (PARK) apply(pend_t);
            else apply_frag(pend_t);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (k == 1) RSTAMP(38);
        issue_taps(k * 6 + 4);
#elif defined(RCAB_APPLY_FIRST)
        if (k == 1) RSTAMP(38);
        if (pend_t >= 0) {                          // residual loads not queued behind the taps
            if constexpr (PARK) {
                load_x(pend_t);
                apply(pend_t);
            } else {
                load_x_frag(pend_t);
                apply_frag(pend_t);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        issue_taps(k * 6 + 4);
#else
        issue_taps(k * 6 + 4);
        if (k == 1) RSTAMP(38);
        if (pend_t >= 0) {
            if constexpr (PARK) {
                load_x(pend_t);
                apply(pend_t);
            } else {
                load_x_frag(pend_t);
                apply_frag(pend_t);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#endif
        if (k == 1) RSTAMP(39);
#ifdef RCAB_Z1_LDS
        if (d.z1) {
            // z1 out of the x-halo buffer: wave w copies exactly the 1-KB pieces it refills by
            // DMA below (i = w, w + 8, ..), so no other wave's halo DMA can overwrite a piece
            // before its copy has read it; 64 lanes = 8 whole pixels (1 KB contiguous)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = (wave + 8 * j) * 8 + (lane >> 3), c = lane & 7, zc = px & 15;
                const uint4 v = *(const uint4*)(xh + px * 128 + ((c ^ (zc & 7)) << 4));
                const size_t o = ((size_t)(b * H + h0 + (px >> 4)) * W + w0 + zc) * 128 + c * 16;
                *(uint4*)((char*)d.z1 + o) = v;
            }
        }
#endif
#ifndef RCAB_A1_MASKED
        if (d.a1) {
            // training copy of a1: the tile's 16x16 interior straight from the a1 image in LDS
            // (complete since the phase-3 barrier), 16-B lanes over whole 2-KB pixel rows, instead
            // of exec-masked 8-B fragment stores from the conv1 epilogue.  Issued before the
            // halo DMA so phase 4's vmcnt(#halo pieces) still leaves only the halo in flight.
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int idx = j * 512 + tid, px = idx >> 3, c = idx & 7;
                const int ar = 1 + (px >> 4), ac = 1 + (px & 15);
                const uint4 v = *(const uint4*)(a1s + (ar * A1W + ac) * 128 + ((c ^ (ac & 7)) << 4));
                const size_t o = ((size_t)(b * H + h0 + (px >> 4)) * W + w0 + (px & 15)) * 128 + c * 16;
                *(uint4*)((char*)d.a1 + o) = v;
            }
        }
#endif
        const bool halo_next = k + 1 < nmine;
        if (halo_next) issue_halo(t + nslot);       // conv1 is done with xh / eh
        if (k == 1) RSTAMP(40);
        // ================= conv2: phases 3..5 =================
        f32x4 acc2[2][4];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n) acc2[m][n] = zero4();
#pragma unroll 1
        for (int p = 3; p < 6; ++p) {
            const int P = k * 6 + p;
            if (p > 3) {
                if (k < 2 && p == 4) RSTAMP(10 + k * 14);
                if (p == 4 && halo_next) {
                    if (wave < (XH_DMA + EH_DMA) % 8) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HALO_W + 1) : "memory");
                    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HALO_W) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (k < 2 && p == 4) RSTAMP(11 + k * 14);
                if (!(k + 1 == nmine && p == 5)) issue_taps(P + 1);
            }
            const char* tapp[3] = {ring + (P & 1) * 3 * TAP_BYTES, ring + (P & 1) * 3 * TAP_BYTES + TAP_BYTES,
                                   ring + (P & 1) * 3 * TAP_BYTES + 2 * TAP_BYTES};
            if (k == 1 && p == 4) RSTAMP(41);
            conv2_phase<T>(acc2, a1s, tapp, p - 3, wr, arow2, q, c16);
            if (k == 1) RSTAMP(42 + (p - 3));
        }
        if (k == 0) RSTAMP(29);
        // ---- conv2 epilogue: t = acc + b2 (parked or carried), pool partial, arrival
        float ps[2][4];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float4 bb = *(const float4*)(cst + 128 + wc * 32 + m * 16 + 4 * q);
            const float bia[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) ps[m][r] = 0.f;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc2[m][n][r] += bia[r];
                    ps[m][r] += acc2[m][n][r];
                }
#ifdef RCAB_PARK_NOSHFL
                if constexpr (PARK) {
                    const size_t o = ((size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16) * 64 + wc * 32 + m * 16 + 4 * q;
                    float v[4] = {acc2[m][n][0], acc2[m][n][1], acc2[m][n][2], acc2[m][n][3]};
                    st4<T>((char*)tpark + o * 2, v);
                }
#endif
            }
        }
#ifndef RCAB_PARK_NOSHFL
        if constexpr (PARK) {                         // t parked with the paired-lane 16-B stores
            const bool odd = q & 1;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                uint2 pk[2];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    pk[m].x = (unsigned)to16<T>(acc2[m][n][0]) | ((unsigned)to16<T>(acc2[m][n][1]) << 16);
                    pk[m].y = (unsigned)to16<T>(acc2[m][n][2]) | ((unsigned)to16<T>(acc2[m][n][3]) << 16);
                }
                const uint2 snd = odd ? pk[0] : pk[1];
                uint2 rcv;
                rcv.x = (unsigned)__shfl_xor((int)snd.x, 16, 64);
                rcv.y = (unsigned)__shfl_xor((int)snd.y, 16, 64);
                const uint4 v = odd ? make_uint4(rcv.x, rcv.y, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, rcv.x, rcv.y);
                const size_t px = (size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16;
                *(uint4*)((char*)tpark + (px * 64 + wc * 32 + (odd ? 16 + 4 * (q - 1) : 4 * q)) * 2) = v;
            }
        }
#endif
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float s = group16_sum(ps[m][r]);
                if (c16 == 0) red[wr * 64 + wc * 32 + m * 16 + 4 * q + r] = s;
            }
        if (k < 2) RSTAMP(12 + k * 14);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (k < 2) RSTAMP(13 + k * 14);
        if (wave == 0) {
            // tile partial -> uncached workspace; the arrival is raised at the next tile's
            // phase-1 boundary, once a vmcnt(0) has drained this store (no stall here)
            __hip_atomic_store(part + ((size_t)tile * B + b) * 64 + lane,
                               (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        arrive_f = tile * B + b;
        if constexpr (!PARK) {
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    tcar[m][n].x = (unsigned)to16<T>(acc2[m][n][0]) | ((unsigned)to16<T>(acc2[m][n][1]) << 16);
                    tcar[m][n].y = (unsigned)to16<T>(acc2[m][n][2]) | ((unsigned)to16<T>(acc2[m][n][3]) << 16);
                }
        }
        pend_t = t;
        if (k < 2) RSTAMP(14 + k * 14);
    }
    // the last tile: its gate comes from this round's other tiles
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    arrive();
    RSTAMP(30);
    if (pend_t >= 0) {
        if constexpr (PARK) load_x(pend_t);           // the residual is in flight during the gate
        else load_x_frag(pend_t);
        if (wave == 0) gate_to_lds(pend_t / tpi, pend_t % tpi == 0, 35);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if constexpr (PARK) apply(pend_t);
        else apply_frag(pend_t);
        RSTAMP(31);
    }
    // block 0 advances the epoch once every block has read it (the next launch on the stream
    // cannot start before this block ends)
    if (blockIdx.x == 0 && wave == 0) {
        unsigned it = 0;
        for (;;) {
            bool mine = true;
            for (int i = lane; i < nslot; i += 64) mine &= ld_poll(sflag + i) == ep1;
            if (__all(mine) || ++it >= POLL_MAX) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (lane == 0) {
            if (it >= POLL_MAX) st_flag(err, 1);
            st_flag(epoch, ep1);
        }
    }
#ifdef FEN_STAMPS
    __syncthreads();
    if (d.stamps && lane < 48 && stamp_lds[wave * 48 + lane] != 0u)
        d.stamps[((size_t)blockIdx.x * 8 + wave) * 48 + lane] = stamp_lds[wave * 48 + lane];
#endif
    (void)lflag;
}

}  // namespace

extern "C" size_t fen_rcab_workspace_bytes(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    const size_t nt = (size_t)B * (H / 16) * (W / 16);
    return nt * 64 * sizeof(float) + (nt + MAX_GRID + 2) * sizeof(int);
}

// The one allocation the library makes: the fused RCAB's hand-off workspace must be uncached
// (hipDeviceMallocUncached) so that pollers on other XCDs never read a stale L2 copy.  It is
// zeroed here and the kernel leaves it zeroed.
extern "C" int fen_rcab_workspace_alloc(int B, int H, int W, void** ws) {
    if (!ws) return FEN_EINVAL;
    const size_t n = fen_rcab_workspace_bytes(B, H, W);
    if (n == 0) return FEN_EINVAL;
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, n, hipDeviceMallocUncached) != hipSuccess) return FEN_EHIP;
    if (hipMemset(p, 0, n) != hipSuccess) {
        (void)hipFree(p);
        return FEN_EHIP;
    }
    *ws = p;
    return FEN_OK;
}
// Diagnostic (synchronises the device): after a completed launch of shape (B, H, W) every
// tile flag equals the epoch and the poll-timeout word is 0; returns the number of words
// that break this (0 = healthy), or < 0 on error.
extern "C" int fen_rcab_workspace_status(const void* ws, int B, int H, int W) {
    if (!ws || B <= 0 || H < 16 || W < 16) return FEN_EINVAL;
    const size_t nt = (size_t)B * (H / 16) * (W / 16);
    const size_t n = nt + MAX_GRID + 2;
    int* h = (int*)malloc(n * sizeof(int));
    if (!h) return FEN_EINVAL;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h, (const char*)ws + nt * 64 * sizeof(float), n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) {
        free(h);
        return FEN_EHIP;
    }
    const int ep = h[nt + MAX_GRID];
    int c = ep == 0 ? 1 : 0;
    for (size_t i = 0; i < nt; ++i) c += h[i] != ep;
    c += h[nt + MAX_GRID + 1] != 0;
    free(h);
    return c;
}
extern "C" int fen_rcab_workspace_free(void* ws) {
    if (ws && hipFree(ws) != hipSuccess) return FEN_EHIP;
    return FEN_OK;
}

static int rcab_num_cus() {
    static int ncu = 0;
    if (ncu == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (ncu <= 0) ncu = 256;
    }
    return ncu;
}

extern "C" int fen_rcab_supported(int dtype, int B, int H, int W, int C, int Cr) {
    if ((dtype != FEN_BF16 && dtype != FEN_F16) || C != 64 || Cr <= 0 || Cr > 16 || B <= 0 || H <= 0 || W <= 0 || H % 16 || W % 16)
        return 0;
    if ((size_t)B * H * W * 128 >= (size_t)0x7fff0000) return 0;
    return (H / 16) * (W / 16) <= rcab_num_cus() ? 1 : 0;
}

extern "C" int fen_rcab_fused(const fen_rcab_desc* d, void* stream) {
    if (!d || !d->x || !d->y || !d->w1 || !d->w2 || !d->b1 || !d->b2 || !d->alpha || !d->fc1 || !d->fc2 || !d->s ||
        !d->ws)
        return FEN_EINVAL;
    if (!fen_rcab_supported(d->dtype, d->B, d->H, d->W, d->C, d->Cr)) return FEN_EUNSUPPORTED;
    if ((d->z1 != nullptr) != (d->a1 != nullptr)) return FEN_EINVAL;
    const int ncu = rcab_num_cus();
    const int tpi = (d->H / 16) * (d->W / 16);         // an image's tiles must be co-resident
    const int ntiles = d->B * tpi;
    int grid = (ncu / tpi) * tpi;                      // rounds of whole images
    if (grid > ntiles) grid = ntiles;
    if (grid > MAX_GRID) grid = (MAX_GRID / tpi) * tpi;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_rcab<bf16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, RCAB_LDS);
        (void)hipFuncSetAttribute((const void*)k_rcab<bf16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, RCAB_LDS);
        (void)hipFuncSetAttribute((const void*)k_rcab<f16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, RCAB_LDS);
        (void)hipFuncSetAttribute((const void*)k_rcab<f16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, RCAB_LDS);
        attr = true;
    }
    hipStream_t st = (hipStream_t)stream;
    if (d->dtype == FEN_F16) {
        if (d->t) hipLaunchKernelGGL((k_rcab<f16, true>), dim3(grid), dim3(512), RCAB_LDS, st, *d);
        else hipLaunchKernelGGL((k_rcab<f16, false>), dim3(grid), dim3(512), RCAB_LDS, st, *d);
    } else {
        if (d->t) hipLaunchKernelGGL((k_rcab<bf16, true>), dim3(grid), dim3(512), RCAB_LDS, st, *d);
        else hipLaunchKernelGGL((k_rcab<bf16, false>), dim3(grid), dim3(512), RCAB_LDS, st, *d);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

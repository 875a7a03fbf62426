// RCAB with the SE gate applied by the consumer (reference src/models/blocks.py:135-153,
// ChannelAttention blocks.py:83-92, the RCAB chain of ResidualGroup blocks.py:185-188).
//
// The gate s_j = sigmoid(W2 relu(W1 mean_hw(t_j))) of RCAB j needs the mean of t_j over the
// whole image, i.e. every tile.  Launch j therefore stops at t_j (and its per-tile sums); launch
// j+1 applies the gate while it builds its own input:
//
//   x_j = x_{j-1} + res_scale * s_{j-1} * t_{j-1}        (on the 20x20 halo of each tile)
//   z1 = conv1(x_j) + b1,  a1 = PReLU(z1)                  (18x18: conv2's halo, recomputed)
//   t_j = conv2(a1) + b2,  part_j[b][tile][c] = sum over the tile of t_j
//
// The kernel boundary is the grid-wide hand-off, so blocks never wait on each other: any grid
// size, no co-residency assumption, no spinning, no workspace, graph-replayable.  A chain
// start (tp == NULL) reads x_j directly (LDS-DMA); the chain end is fen_se_fused.
//
// Structure (one 512-thread block per CU, persistent over its tiles, XCD-aware so an image's
// tiles share an L2):
//   * both filters stream tap by tap from L2 through a 6-slot LDS ring (3 taps per phase,
//     refilled one phase ahead): 144 KB of filters do not fit beside the activation images;
//   * the next tile's input is prepared during the current tile's conv2: the x_{j-1} / t_{j-1}
//     halo loads go out right after conv1, and x_j is written into the (then free) halo image
//     after conv2, together with the x_j interior (the next launch's residual base);
//   * conv1 on 21 pixel fragments (18 rows of 16 + 3 fragments of the 2 edge columns, read
//     from a row-keyed copy of halo columns 16..19) -> bias + PReLU -> a1 image in LDS (zero
//     outside the image = conv2's padding); conv2 with the halo-row-reuse MFMA order.
// 16-bit (bf16 / fp16) activations, fp32 MFMA accumulation, C = 64, Cr <= 16.
#include "fen_common.h"

namespace {

constexpr int XW = 20;                       // conv1 input halo, 20x20 px
constexpr int XH_BYTES = XW * XW * 128;      // 51200 = 50 DMA pieces
constexpr int XH_DMA = XH_BYTES / 1024;
constexpr int EH_BYTES = XW * 4 * 128;       // halo columns 16..19 again, row-keyed: 10 pieces
constexpr int EH_DMA = EH_BYTES / 1024;
constexpr int A1W = 18;                      // a1 image = conv2 halo, 18x18, hcol layout
constexpr int A1_BYTES = A1W * A1W * 128;    // 41472
constexpr int TAP_BYTES = 64 * 128;          // one filter tap [64 co][64 ci]
constexpr int MAXG = 16;                     // gates precomputed per block (tiles per block)
constexpr int O_XH = 0;
constexpr int O_EH = O_XH + XH_BYTES;
constexpr int O_A1 = O_EH + EH_BYTES;
constexpr int O_RING = O_A1 + A1_BYTES;
constexpr int O_RED = O_RING + 6 * TAP_BYTES;   // [4][64] f32 pool partials of the 4 row waves
constexpr int O_CST = O_RED + 4 * 64 * 4;       // b1[64] alpha[64] b2[64]
constexpr int O_GATE = O_CST + 3 * 64 * 4;      // [MAXG][64] f32: res_scale * s of each tile's image
#ifdef FEN_STAMPS
constexpr int O_STAMP = O_GATE + MAXG * 64 * 4; // diagnostic build: [8 waves][48] u32 stamps
constexpr int RD_LDS = O_STAMP + 8 * 48 * 4;
#else
constexpr int RD_LDS = O_GATE + MAXG * 64 * 4;
#endif
// prologue scratch inside the (then unused) a1 image: fc1 [16][64], fc2 [64][16] f32 and a
// [8 waves][128] f32 gate workspace
constexpr int O_PFC = O_A1;
constexpr int O_PWS = O_A1 + 2 * 1024 * 4;
static_assert(O_PWS + 8 * 128 * 4 <= O_A1 + A1_BYTES, "prologue scratch");
static_assert(RD_LDS <= 163840, "LDS budget");
static_assert(O_RING % 16 == 0 && O_RED % 16 == 0 && O_GATE % 16 == 0, "alignment");

constexpr int HCH = XW * XW * 8;             // 16-B chunks of the 20x20 halo: 3200
constexpr int HPT = (HCH + 511) / 512;       // per thread: 7 (the 7th for threads < 128: waves 0, 1)
static_assert(HCH - (HPT - 1) * 512 == 128, "the last halo chunk row is waves 0 and 1 exactly");

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

// 16-B chunk position in the edge image: pixel e = row*4 + col', key = (2 row) & 7 (checked
// against ds_read_b128's lane groups for every edge fragment, kh, kw, k-half: conflict-free)
__device__ __forceinline__ int ekey_of(int row) { return (2 * row) & 7; }
__device__ __forceinline__ int ekey(int row, int chunk) { return (chunk ^ ekey_of(row)) << 4; }

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

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
// halo-row-reuse order: per k-half the wave loads its NR + 2 input rows once and reuses them
// across the 3 kernel rows.  Slots 0..NR-1 are main rows row0.. (16 columns); without MAIN4
// slot 4 is edge fragment eidx4, with HAS5 slot 5 is edge fragment 1 (edge reads do not reuse
// across kh: their lanes map to (row, column)).
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
    // opaque lane coordinates: addresses are recomputed per phase instead of being hoisted out
    // of the tile loop (loop-invariant offsets live through conv2, the register peak, spill)
    asm volatile("" : "+v"(c16), "+v"(arow), "+v"(q));
    // (an explicitly software-pipelined form -- the next (k-half, m) group's fragments read during
    // the current group's MFMAs -- measured no faster per phase and pushed the deferred kernel
    // into spills: 33.0 -> 35.8 us per launch)
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
    }
}

// vmcnt with an immediate chosen from a small runtime value (wave-uniform)
__device__ __forceinline__ void vm_wait(int n) {
    switch (n) {
#define RD_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        RD_VMC(1) RD_VMC(2) RD_VMC(3) RD_VMC(4) RD_VMC(5) RD_VMC(6) RD_VMC(7) RD_VMC(8) RD_VMC(9) RD_VMC(10)
        RD_VMC(11) RD_VMC(12) RD_VMC(13) RD_VMC(14) RD_VMC(15) RD_VMC(16) RD_VMC(17) RD_VMC(18) RD_VMC(19)
        RD_VMC(20) RD_VMC(21) RD_VMC(22) RD_VMC(23) RD_VMC(24)
#undef RD_VMC
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// kernel arguments: the forward descriptor, plus the backward form's operands
struct RdArgs {
    fen_rcab_deferred_desc d;
    // BWD: the RCAB's data gradient through both convs (see fen_rcab_bwd): d.x = dt,
    // d.w1 / d.w2 = conv2 / conv1 mode-2 packs, d.alpha, d.t = dx out, d.part = the DOT
    // partials (or NULL)
    const void* z1;            // saved conv1 pre-activation
    void* dz1;                 // out: dz1 (conv1's weight-gradient operand)
    float* dpart;              // out: per-tile PReLU slope-gradient partials
    const void* dy;            // added to dx (the RCAB's output gradient)
    const void* dot_t;         // t of the next RCAB backward (with d.part)
    // GC: the group conv (d.w2 / d.b2 = its pack and bias, d.t = its output) + this residual
    const void* gres;
    // SEB: the SE backward folded in -- d.x = dy (the halo source), d.pp = the DOT partials
    // [B][tiles][64], A.se_s / d.pmean / d.phid the saved s / mean / hid, d.pfc1 / d.pfc2 the
    // FC weights, d.xo = dt out; FC weight-gradient rows per image
    const float* se_s;
    float* se_dw1p;
    float* se_dw2p;
};

// ------------------------------------------------------------------------------------
// the kernel.  DEFER: the input is (x_{j-1}, t_{j-1}, part_{j-1}) and the gate is applied
// while building the halo; else x_j is read directly.  TRAIN: z1 / a1 copies for the backward.
// ------------------------------------------------------------------------------------
// BWD (DEFER = TRAIN = false): the RCAB backward's two data gradients in one launch, the
// same tile pipeline on transposed filters -- dz1 = conv2^T(dt) on the 18x18 halo, times the
// PReLU derivative at the saved z1 (its 18x18 halo DMA'd into the a1 image, then overwritten
// in place by dz1; slope-gradient partials over the tile interior), dx = conv1^T(dz1) +
// dy (+ the tile sums of dx * t_next for the next SE backward).
// SEB (with BWD): the SE backward and its apply folded into the input path -- every block
// recomputes its tiles' images' SE backward in the prologue (k_se_bwd_fused's arithmetic and
// order) and the DMA'd dy halo becomes dt = dy * rs * s + g in place (zero outside the image),
// the tile's own dt going out for conv2's weight gradient: no separate dt pass over HBM.
// GC (DEFER, not TRAIN): a ResidualGroup's end -- the last RCAB's gate and scaled residual
// applied while building the input (straight into the a1 image, 18x18), then the group conv
// (one 3x3 conv on the conv2 path) + bias + the group's residual (blocks.py:185-189): the
// chain end's separate gate/apply launch and its tensor round trip disappear.
template <typename T, bool DEFER, bool TRAIN, bool BWD = false, bool GC = false, bool SEB = false>
__global__ __launch_bounds__(512, 1) void k_rcab_d(const RdArgs A) {
    const fen_rcab_deferred_desc& d = A.d;
    static_assert(!(BWD && (DEFER || TRAIN)), "the backward form is its own mode");
    static_assert(!GC || (DEFER && !TRAIN && !BWD), "the group end is a deferred single conv");
    static_assert(!SEB || BWD, "the SE backward folds into the backward form");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* xh = smem + O_XH;
    char* eh = smem + O_EH;
    char* a1s = smem + O_A1;
    char* ring = smem + O_RING;
    float* red = (float*)(smem + O_RED);
    float* cst = (float*)(smem + O_CST);
    float* gate = (float*)(smem + O_GATE);
#ifdef FEN_STAMPS
    unsigned* stamp_lds = (unsigned*)(smem + O_STAMP);
    for (int i = threadIdx.x; i < 8 * 48; i += blockDim.x) stamp_lds[i] = 0u;
    __syncthreads();
#endif

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: per-wave roles are scalar branches
    const int q = lane >> 4, c16 = lane & 15;
    // conv1: channel half, fragment group.  The groups with edge fragments (g = 2, 3: the most
    // reads and MFMAs) run on waves 0-3, which win the issue arbitration against their SIMD
    // partners (waves 4-7, MI355X_MICROARCH.md 'Two waves per SIMD'): 34.0 -> 33.0 us per launch
    const int ch = wave & 1, g = (wave >> 1) ^ 2;
    const int wr = wave >> 1, wc = wave & 1;         // conv2: row group, channel half
    const int H = d.H, W = d.W, B = d.B;
    const int twn = W >> 4, tpi = twn * (H >> 4);
    const int ntiles = B * tpi;
    const int nslot = gridDim.x;
    // XCD-aware slot: an image's tiles (consecutive slots) on one XCD, so neighbouring tiles'
    // halo rows come from that XCD's L2.  Any permutation is correct (blocks are independent).
    const int slot = xcd_block();
    const int nmine = (ntiles - slot + nslot - 1) / nslot;

    const size_t act_bytes = (size_t)B * H * W * 128;
    const i32x4 xr4 = make_rsrc(d.x, (unsigned)act_bytes);
    const i32x4 w1r = make_rsrc(d.w1, 9u * 64u * 128u);
    const i32x4 w2r = make_rsrc(d.w2, 9u * 64u * 128u);
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(DEFER ? d.tp : d.x), 0, (int)act_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc((void*)d.xo, 0, d.xo ? (int)act_bytes : 0, 0x00020000);

    // ring: phase P of the block's sequence (6 per tile) uses slots (P & 1) * 3 + i.
    // phase p = 0..2: conv1 taps 3p..3p+2 column-wise; p = 3..5: conv2 taps (kh, kw = p - 3)
    auto issue_taps = [&](int P) {
        const int p = GC ? P % 3 + 3 : P % 6;   // GC: three phases per tile, all on w2
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
    // x halo (20x20, hcol key) + edge copy (halo columns 16..19, row key) by LDS-DMA; deferred
    // mode DMAs x_{j-1} without the edge copy (the combine writes both from registers)
    constexpr int NDMA = (DEFER || SEB) ? XH_DMA : XH_DMA + EH_DMA;
    auto issue_halo = [&](int t) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        for (int i = wave; i < NDMA; i += 8) {
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
    const int ndma = (NDMA / 8) + (wave < NDMA % 8 ? 1 : 0);   // this wave's halo pieces
    // deferred: the tile's t_{j-1} halo chunks into registers (out of range = 0 = the zero
    // padding); chunk i = tid + 512 j is pixel i >> 3, 16-B channel chunk i & 7
    const int nch = wave < 2 ? HPT : HPT - 1;          // this wave's halo chunks (wave-uniform)
    // (the chunk registers are declared per tile by the caller: a tv[] that outlives the tile
    // loop body stays live through conv1, the register peak)
    auto load_t = [&](int t, uint4 (&tv)[HPT]) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        int tq = tid;
        asm volatile("" : "+v"(tq));   // opaque: per-chunk addresses are not hoisted out of the tile loop
#pragma unroll
        for (int j = 0; j < HPT; ++j) {
            if (j == HPT - 1 && wave >= 2) break;
            const int i = tq + 512 * j, p = i >> 3, c = i & 7;
            const int hr = p / XW, hc = p - hr * XW;
            const int gh = h0 - 2 + hr, gw = w0 - 2 + hc;
            const int off = ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W)
                                ? (((b * H + gh) * W + gw) * 64 + c * 8) * 2 : 0x7ffffff0;
            tv[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(trs, off, 0, 0));
        }
    };
    // BWD: the saved z1's 18x18 halo into the a1 image (its layout; zero outside the image).
    // 41 pieces, the last one half: its upper 32 lanes are exec-masked off (no LDS write past
    // the image, which ends where the filter ring starts)
    const i32x4 zr4 = make_rsrc(BWD ? A.z1 : d.x, (unsigned)act_bytes);
    auto issue_z1 = [&](int t) {
        constexpr int ZCH = A1W * A1W * 8, ZDMA = (ZCH + 63) / 64;
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        for (int i = wave; i < ZDMA; i += 8) {
            const int L = i * 64 + lane, P = L >> 3;
            const int ar = P / A1W, ac = P - ar * A1W;
            const int c = (L & 7) ^ (ac & 7);
            const int gh = h0 - 1 + ar, gw = w0 - 1 + ac;
            const int voff = ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W)
                                 ? (((b * H + gh) * W + gw) * 64 + c * 8) * 2 : 0x7ffffff0;
            if (L < ZCH) dma16(zr4, __builtin_amdgcn_readfirstlane(lds_addr(a1s + i * 1024)), voff);
        }
    };
    // x_j = x_{j-1} (DMA'd halo image) + (res_scale s) t_{j-1}, in place, + the edge copy and,
    // for the tile's own 16x16 pixels, x_j out (buffer stores: the halo ring's offsets fall out
    // of range and are dropped, so every wave issues exactly nch stores).  Each thread rewrites
    // only its own chunks; the DMA'd bytes came from other waves: a barrier precedes this.
    auto combine_halo = [&](int t, int k, const uint4 (&tv)[HPT]) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        // this thread's 8 channels (c = tid & 7 for every chunk): the gate in registers once
        const float* sv = gate + (k % MAXG) * 64 + (tid & 7) * 8;
        const float4 s0 = *(const float4*)sv, s1 = *(const float4*)(sv + 4);
        const float s8[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        int tq = tid;
        asm volatile("" : "+v"(tq));   // opaque: per-chunk addresses are not hoisted out of the tile loop
#pragma unroll
        for (int j = 0; j < HPT; ++j) {
            if (j == HPT - 1 && wave >= 2) break;
            const int i = tq + 512 * j, p = i >> 3, c = i & 7;
            const int hr = p / XW, hc = p - hr * XW;
            char* px = xh + hr * (XW * 128) + hcol(hc, c);
            float xf[8], tf[8], y[8];
            unpack16<T>(*(const uint4*)px, xf);
            unpack16<T>(tv[j], tf);
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = tf[e] * s8[e] + xf[e];
            const uint4 v = pack16<T>(y);
            if constexpr (GC) {
                if ((unsigned)(hr - 1) < 18u && (unsigned)(hc - 1) < 18u)
                    *(uint4*)(a1s + (hr - 1) * (A1W * 128) + hcol(hc - 1, c)) = v;
            } else {
                *(uint4*)px = v;
                if (hc >= 16) *(uint4*)(eh + (hr * 4 + (hc - 16)) * 128 + ekey(hr, c)) = v;
            }
            const bool own = (unsigned)(hr - 2) < 16u && (unsigned)(hc - 2) < 16u;
            const int off = own ? (((b * H + h0 - 2 + hr) * W + w0 - 2 + hc) * 64 + c * 8) * 2 : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), ors, off, 0, 0);
        }
    };
    // SEB: dt = dy * rs * s + g over the DMA'd dy halo image in place (+ the edge copy; zero
    // outside the image), the tile's own dt out (nch buffer stores per wave, as combine_halo)
    auto se_halo = [&](int t, int k) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const float rs = d.res_scale;
        // this thread's 8 channels (c = tid & 7 for every chunk): s and g in registers once
        float s8[8], g8[8];
        {
            const float* sv = gate + (4 + 2 * k) * 64 + (tid & 7) * 8;
            const float4 s0 = *(const float4*)sv, s1 = *(const float4*)(sv + 4);
            const float4 g0 = *(const float4*)(sv + 64), g1 = *(const float4*)(sv + 68);
            s8[0] = s0.x, s8[1] = s0.y, s8[2] = s0.z, s8[3] = s0.w, s8[4] = s1.x, s8[5] = s1.y, s8[6] = s1.z, s8[7] = s1.w;
            g8[0] = g0.x, g8[1] = g0.y, g8[2] = g0.z, g8[3] = g0.w, g8[4] = g1.x, g8[5] = g1.y, g8[6] = g1.z, g8[7] = g1.w;
        }
        int tq = tid;
        asm volatile("" : "+v"(tq));
#pragma unroll
        for (int j = 0; j < HPT; ++j) {
            if (j == HPT - 1 && wave >= 2) break;
            const int i = tq + 512 * j, p = i >> 3, c = i & 7;
            const int hr = p / XW, hc = p - hr * XW;
            const int gh = h0 - 2 + hr, gw = w0 - 2 + hc;
            const bool in = (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
            char* px = xh + hr * (XW * 128) + hcol(hc, c);
            float xf[8], y[8];
            unpack16<T>(*(const uint4*)px, xf);
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = in ? xf[e] * rs * s8[e] + g8[e] : 0.f;
            const uint4 v = pack16<T>(y);
            *(uint4*)px = v;
            if (hc >= 16) *(uint4*)(eh + (hr * 4 + (hc - 16)) * 128 + ekey(hr, c)) = v;
            const bool own = (unsigned)(hr - 2) < 16u && (unsigned)(hc - 2) < 16u;
            const int off = own ? (((b * H + gh) * W + gw) * 64 + c * 8) * 2 : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), ors, off, 0, 0);
        }
    };

    // the per-channel constants, loaded before the start-up DMA and written to LDS after its
    // wait (read right after the DMA issue, their use made the compiler wait for the DMA too)
    float cb1 = 0.f, cal = 0.f, cb2 = 0.f;
    if (tid < 64) {
        if (!BWD) cb1 = d.b1[tid];
        if (!GC) cal = d.alpha[tid];   // (the group conv has no PReLU: d.alpha unset)
        if (!BWD) cb2 = d.b2[tid];
    }
    // DEFER: the gate chain's operands (the SE weights, the first 16 tile partials of this
    // wave's first tile) before the start-up DMA, so they return first
    float f1e[2] = {0.f, 0.f}, f2e[2] = {0.f, 0.f}, v0e[16];
    if constexpr (DEFER) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int i = tid + r * 512, c = i >> 4, j = i & 15;
            f1e[r] = i < d.Cr * 64 ? d.pfc1[i] : 0.f;
            f2e[r] = j < d.Cr ? d.pfc2[c * d.Cr + j] : 0.f;
        }
        const int b = (slot + (wave < nmine ? wave : 0) * nslot) / tpi;
        const float* pp = d.pp + (size_t)b * tpi * 64 + lane;
#pragma unroll
        for (int u = 0; u < 16; ++u) v0e[u] = pp[(size_t)(u < tpi ? u : tpi - 1) * 64];
    }
    // SEB: the SE backward's operands of this wave's tile (wave k < nmine <= 6 handles tile k)
    float w2v[16], w1v[16], hv[16], sp[16], sv = 0.f, mv = 0.f;
    auto seb_loads = [&]() {
        if (wave < nmine) {
            const int Cr = d.Cr, b = (slot + wave * nslot) / tpi;
            const float* pp = d.pp + (size_t)b * tpi * 64 + lane;
#pragma unroll
            for (int u = 0; u < 16; ++u) sp[u] = pp[(size_t)(u < tpi ? u : tpi - 1) * 64];   // (unconditional: no early wait)
            sv = A.se_s[(size_t)b * 64 + lane];
#pragma unroll
            for (int j = 0; j < 16; ++j) w2v[j] = d.pfc2[lane * Cr + (j < Cr ? j : Cr - 1)];
#pragma unroll
            for (int j = 0; j < 16; ++j) hv[j] = d.phid[(size_t)b * Cr + (j < Cr ? j : Cr - 1)];
#pragma unroll
            for (int j = 0; j < 16; ++j) w1v[j] = d.pfc1[(j < Cr ? j : Cr - 1) * 64 + lane];
            mv = d.pmean[(size_t)b * 64 + lane];
        }
    };
    // ---- start-up: first taps and the first halo go out before anything else waits on memory
    uint4 tv0[HPT];
    issue_taps(0);
    issue_halo(slot);
    if constexpr (BWD) issue_z1(slot);
    if constexpr (DEFER) load_t(slot, tv0);
    if constexpr (DEFER) {
        // the gates of this block's tiles (<= MAXG): wave w handles tiles w, w + 8; lane c sums
        // the image's tile partials in tile order (every block computes identical values), then
        // FC1 -> ReLU -> FC2 -> sigmoid through the wave's LDS scratch
        float* fcs = (float*)(smem + O_PFC);
        const int Cr = d.Cr;
        // the first 16 tile partials of this wave's first tile go out before the SE weights'
        // round trip through LDS, so the two latencies overlap (one round trip, not two)
        float v0[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v0[u] = u < tpi ? v0e[u] : 0.f;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            fcs[tid + r * 512] = f1e[r];
            fcs[1024 + tid + r * 512] = f2e[r];
        }
        __syncthreads();
        float* ws = (float*)(smem + O_PWS) + wave * 128;
        for (int k = wave; k < nmine; k += 8) {
            const int t = slot + k * nslot, b = t / tpi;
            const float* pp = d.pp + (size_t)b * tpi * 64 + lane;
            // 16 tile partials in flight per lane (a dependent chain of loads took ~4 us), summed
            // in tile order
            float m = 0.f;
            for (int i0 = 0; i0 < tpi; i0 += 16) {
                float v[16];
                if (i0 == 0 && k == wave) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = v0[u];
                } else {
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = i0 + u < tpi ? pp[(size_t)(i0 + u) * 64] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) m += v[u];
            }
            const float mean = m * d.inv_hw;
            ws[lane] = mean;
            const int j = lane & 15, part4 = lane >> 4;
            float h = 0.f;
#pragma unroll
            for (int c = 0; c < 16; c += 4) {
                const float4 w = *(const float4*)(fcs + j * 64 + part4 * 16 + c);
                const float4 mv = *(const float4*)(ws + part4 * 16 + c);
                h += w.x * mv.x + w.y * mv.y + w.z * mv.z + w.w * mv.w;
            }
            h += __shfl_xor(h, 16, 64);
            h += __shfl_xor(h, 32, 64);
            const float hid = fmaxf(h, 0.f);                 // hidden unit j (0 for j >= Cr)
            if (lane < 16) ws[64 + lane] = hid;
            float z = 0.f;
#pragma unroll
            for (int c = 0; c < 16; c += 4) {
                const float4 w = *(const float4*)(fcs + 1024 + lane * 16 + c);
                const float4 hv = *(const float4*)(ws + 64 + c);
                z += w.x * hv.x + w.y * hv.y + w.z * hv.z + w.w * hv.w;
            }
            const float sg = 1.f / (1.f + expf(-z));
            gate[k * 64 + lane] = sg * d.res_scale;
            if (t % tpi == 0) {                              // the user-visible copies, once per image
                if (d.ps) d.ps[(size_t)b * 64 + lane] = sg;
                if (d.pmean) d.pmean[(size_t)b * 64 + lane] = mean;
                if (d.phid && lane < Cr) d.phid[(size_t)b * Cr + lane] = hid;
            }
        }
    }
    if constexpr (SEB) {
        // the SE backward of each of this block's tiles' images (<= 6 tiles: gate rows 4..15;
        // rows 0..3 hold the slope partials): wave w handles tiles w (< 6), lane = channel c,
        // in k_se_bwd_fused's order -- quarter sums over partials q, q+4, ..., their fixed-order
        // combine, FC2^T by wave sums, FC1^T in hidden-unit order
        // (nmine <= 6: wave k handles tile k.  Its operands are loaded here, behind the
        // start-up DMA: issued before it they measured 0.2% slower on the training step)
        seb_loads();
        const int Cr = d.Cr;
        if (wave < nmine) {
            const int k = wave;
            const int t = slot + k * nslot, b = t / tpi;
            const float* pp = d.pp + (size_t)b * tpi * 64 + lane;
            float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (u < tpi) a4[u & 3] += sp[u];
            for (int i0 = 16; i0 < tpi; i0 += 16) {
                float v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = i0 + u < tpi ? pp[(size_t)(i0 + u) * 64] : 0.f;
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (i0 + u < tpi) a4[u & 3] += v[u];
            }
            const float a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
            const float dz = a * d.res_scale * sv * (1.f - sv);
            float dh[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                dh[j] = 0.f;
                dh[j] += w2v[j] * dz;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
                for (int j = 0; j < 16; ++j) dh[j] += __shfl_xor(dh[j], o, 64);
#pragma unroll
            for (int j = 0; j < 16; ++j) dh[j] = j < Cr && hv[j] > 0.f ? dh[j] : 0.f;
            float ga = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (j < Cr) ga += w1v[j] * dh[j];
            gate[(4 + 2 * k) * 64 + lane] = sv;
            gate[(5 + 2 * k) * 64 + lane] = ga * d.inv_hw;
            if (t % tpi == 0) {                              // the FC weight-gradient rows, once per image
                float* w2p = A.se_dw2p + (size_t)b * 64 * Cr;
                float* w1p = A.se_dw1p + (size_t)b * 64 * Cr;
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (j < Cr) {
                        w2p[lane * Cr + j] = dz * hv[j];
                        w1p[j * 64 + lane] = dh[j] * mv;
                    }
            }
        }
    }
    RSTAMP(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < 64) {
        cst[tid] = cb1;
        cst[64 + tid] = cal;
        cst[128 + tid] = cb2;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (DEFER) {
        combine_halo(slot, 0, tv0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                         // a1 scratch and the halo image
    }
    if constexpr (SEB) {
        se_halo(slot, 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    RSTAMP(1);

    if constexpr (GC) {
        // ---- the group conv on the a1 image (the combine wrote y there), 3 tap phases per
        // tile; the next tile's x / t go out at phase 1 into the free halo image / registers
        const int arow2 = wc * 32 + c16;
        const int nst_gc = 4 + nch;                      // out stores + the combine's y stores
#pragma unroll 1
        for (int k = 0; k < nmine; ++k) {
            const int t = slot + k * nslot;
            const int b = t / tpi, tile = t - b * tpi;
            const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
            const bool next = k + 1 < nmine;
            f32x4 acc2[2][4];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc2[m][n] = zero4();
            uint2 rv[2][4];
            uint4 tv[HPT];
            int nhalo = 0;
#pragma unroll 1
            for (int p = 0; p < 3; ++p) {
                const int P = k * 3 + p;
                if (p > 0 || k > 0) {
                    if (p == 0) vm_wait(nst_gc);         // this phase's taps; the last tile's stores drain on
                    else if (p == 1) vm_wait(8);         // this phase's taps; the residual loads may trail
                    else vm_wait(nhalo);                 // this phase's taps; the next halo stays in flight
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                }
                if (p < 2 || next) issue_taps(P + 1);
                if (p == 0) {
#pragma unroll
                    for (int m = 0; m < 2; ++m)
#pragma unroll
                        for (int n = 0; n < 4; ++n) {
                            const size_t o = ((size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16) * 64 + wc * 32 + m * 16 + 4 * q;
                            rv[m][n] = *(const uint2*)((const char*)A.gres + o * 2);
                        }
                }
                if (p == 1 && next) {
                    issue_halo(t + nslot);
                    load_t(t + nslot, tv);
                    nhalo = ndma + nch;
                }
                const char* tapp[3] = {ring + (P & 1) * 3 * TAP_BYTES, ring + (P & 1) * 3 * TAP_BYTES + TAP_BYTES,
                                       ring + (P & 1) * 3 * TAP_BYTES + 2 * TAP_BYTES};
                conv2_phase<T>(acc2, a1s, tapp, p, wr, arow2, q, c16);
            }
            // ---- out = conv + bias + the group's residual (paired-lane 16-B stores)
            const bool odd = q & 1;
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const float4 bb = *(const float4*)(cst + 128 + wc * 32 + m * 16 + 4 * q);
                const float bia[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    acc2[m][n][0] += bia[0] + lo16<T>(rv[m][n].x);
                    acc2[m][n][1] += bia[1] + hi16<T>(rv[m][n].x);
                    acc2[m][n][2] += bia[2] + lo16<T>(rv[m][n].y);
                    acc2[m][n][3] += bia[3] + hi16<T>(rv[m][n].y);
                }
            }
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                uint2 pk[2];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    pk[m].x = pack2<T>(acc2[m][n][0], acc2[m][n][1]);
                    pk[m].y = pack2<T>(acc2[m][n][2], acc2[m][n][3]);
                }
                const uint2 snd = odd ? pk[0] : pk[1];
                uint2 rcv;
                rcv.x = (unsigned)__shfl_xor((int)snd.x, 16, 64);
                rcv.y = (unsigned)__shfl_xor((int)snd.y, 16, 64);
                const uint4 v = odd ? make_uint4(rcv.x, rcv.y, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, rcv.x, rcv.y);
                const size_t px = (size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16;
                *(uint4*)((char*)d.t + (px * 64 + wc * 32 + (odd ? 16 + 4 * (q - 1) : 4 * q)) * 2) = v;
            }
            if (next) {
                // the next halo (DMA + t chunks) landed in every wave; the next taps (3) and the
                // out stores (4) stay in flight; everyone is past phase 2's reads of the a1 image
                asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                combine_halo(t + nslot, k + 1, tv);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }

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
        a1o4[m] = ar4 <= 17 ? (ar4 * A1W + ac4) * 128 + ((chunk ^ (ac4 & 7)) << 4) + (q & 1) * 8
                            : (O_RED - O_A1) + 4 * 64 * 4 - 16;   // pad lanes: a dummy word (red's last row)
        a1o5[m] = (ar5 * A1W + ac5) * 128 + ((chunk ^ (ac5 & 7)) << 4) + (q & 1) * 8;
    }
    // output stores this wave issues after the next tile's first taps (t and, for wave 0, the
    // tile's partial row; deferred: + the x_j chunks): the phase-0 wait leaves them in flight.
    // (Without DEFER the next halo's DMA is older than those taps: waited for as well.)
    const int nst_tail = 4 + ((wave == 0 && d.part) ? 1 : 0) + ((DEFER || SEB) ? nch : 0);

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
                if (p == 0) vm_wait(nst_tail);           // this phase's taps landed; last tile's stores drain on
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (k < 2) RSTAMP(3 + k * 14 + p * 2);
            }
            issue_taps(P + 1);
            if constexpr (BWD) {
                if (p == 0 && k > 0) issue_z1(t);   // the a1 image is free since the last barrier
            }
            const char* tapp[3] = {ring + (P & 1) * 3 * TAP_BYTES, ring + (P & 1) * 3 * TAP_BYTES + TAP_BYTES,
                                   ring + (P & 1) * 3 * TAP_BYTES + 2 * TAP_BYTES};
            if (g < 2) conv1_kw<T, true, false>(acc1, xh, eh, tapp, p, c16, row0, eidx4, arow1, q);
            else if (g == 2) conv1_kw<T, false, false>(acc1, xh, eh, tapp, p, c16, row0, eidx4, arow1, q);
            else conv1_kw<T, false, true>(acc1, xh, eh, tapp, p, c16, row0, eidx4, arow1, q);
        }
        if (k < 2) RSTAMP(8 + k * 14);
        // ---- conv1 epilogue: bias + PReLU -> a1 image (zero outside the image; branch-free,
        //      precomputed offsets); training: z1 interior with paired-lane 16-B stores
        {
            const bool colok = (unsigned)(w0 - 1 + c16) < (unsigned)W;
            const bool ok4 = (unsigned)(h0 - 1 + ar4) < (unsigned)H && (unsigned)(w0 - 1 + ac4) < (unsigned)W;
            const bool ok5 = (unsigned)(h0 - 1 + ar5) < (unsigned)H && (unsigned)(w0 - 1 + ac5) < (unsigned)W;
            float zs[2][6][4];
            if constexpr (BWD) {
                // dz1 = conv2^T(dt) * PReLU'(z1) (zero outside the image = conv1^T's padding),
                // in place over the DMA'd z1; slope partials over the tile interior
                float dal[2][4];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const float4 aa = *(const float4*)(cst + 64 + ch * 32 + m * 16 + 4 * q);
                    const float alp[4] = {aa.x, aa.y, aa.z, aa.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) dal[m][r] = 0.f;
#pragma unroll
                    for (int f = 0; f < 6; ++f) {
                        if (!(f < 5 || has5)) continue;
                        bool ok;
                        if (f < 4) ok = colok && (unsigned)(h0 - 1 + row0 + f) < (unsigned)H;
                        else ok = f == 4 ? ok4 : ok5;
                        const int ar = f < 4 ? row0 + f : f == 4 ? ar4 : ar5;
                        const int ac = f < 4 ? c16 : f == 4 ? ac4 : ac5;
                        const bool inner = ok && (unsigned)(ar - 1) < 16u && (unsigned)(ac - 1) < 16u;
                        const float okf = ok ? 1.f : 0.f;
                        const int off = f < 4 ? a1m[m] + f * (A1W * 128) : f == 4 ? a1o4[m] : a1o5[m];
                        float z[4], a[4];
                        ld4<T>(a1s + off, z);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float v = acc1[m][f][r];
                            a[r] = okf * prelu_bwd_f(v, z[r], alp[r]);
                            zs[m][f][r] = a[r];
                            if (inner) dal[m][r] += prelu_dalpha_f(v, z[r]);
                        }
                        st4<T>(a1s + off, a);
                    }
                }
                // per-channel sums of this wave's fragment group -> its row of the (otherwise
                // unused) gate area; combined in a fixed order after the phase-3 barrier
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float sm = group16_sum(dal[m][r]);
                        if (c16 == 0) gate[g * 64 + ch * 32 + m * 16 + 4 * q + r] = sm;
                    }
            } else {
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
            }
            if constexpr (TRAIN || BWD) {
                void* zout = BWD ? A.dz1 : d.z1;
                // interior pixels only (a1 rows / cols 1..16): lanes q and q^1 (same pixel) trade
                // one 4-channel half so each store is 16 B
                const bool odd = q & 1;
#pragma unroll
                for (int f = 0; f < 6; ++f) {
                    uint2 pk[2];
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        pk[m].x = pack2<T>(zs[m][f][0], zs[m][f][1]);
                        pk[m].y = pack2<T>(zs[m][f][2], zs[m][f][3]);
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
                    *(uint4*)((char*)zout + o * 2) = v;
                }
            }
        }
        // ---- phase-3 boundary: the a1 image is complete; the halo image is free
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (k < 2) RSTAMP(9 + k * 14);
        // (issuing them before the conv1 epilogue behind an extra barrier measured slower:
        // 34.0 -> 34.3 us per launch; the LDS-DMA of a phase's taps takes ~1.1-1.4 us to land,
        // so conv2's 0.64-us phases 4 and 5 wait ~0.7 us each)
        if constexpr (BWD) {
            // (stored before taps(4): the phase-4 wait covers it)
            if (wave == 0)
                A.dpart[((size_t)b * tpi + tile) * 64 + lane] =
                    (gate[lane] + gate[64 + lane]) + (gate[128 + lane] + gate[192 + lane]);
        }
        issue_taps(k * 6 + 4);
        if constexpr (TRAIN) {
            // a1 for the backward: the tile's 16x16 interior straight from the a1 image, 16-B
            // lanes over whole 2-KB pixel rows (4 stores per thread)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int idx = j * 512 + tid, px = idx >> 3, c = idx & 7;
                const int ar = 1 + (px >> 4), ac = 1 + (px & 15);
                const uint4 v = *(const uint4*)(a1s + (ar * A1W + ac) * 128 + ((c ^ (ac & 7)) << 4));
                const size_t o = ((size_t)(b * H + h0 + (px >> 4)) * W + w0 + (px & 15)) * 128 + c * 16;
                *(uint4*)((char*)d.a1 + o) = v;
            }
        }
        const bool next = k + 1 < nmine;
        // the next tile's input goes out now: LDS-DMA into the free halo image (chain start), or
        // x_{j-1} / t_{j-1} chunks into registers (deferred; combined after conv2)
        int nhalo = 0;                                   // vector-memory ops issued after taps(4)
        uint4 tv[HPT];
        // (issued at phase 5 instead, behind conv2's last taps, the ~1.5 us of DMA / load issue
        // lands in phase 5 and phase 4 waits as long: 36.0 -> 36.8 us per launch)
        if (next) {
            issue_halo(t + nslot);
            nhalo = ndma;
            if constexpr (DEFER) {
                load_t(t + nslot, tv);
                nhalo += nch;
            }
        }
        // BWD: the epilogue's dy / t_next operands, behind the next halo: the phase-4 wait leaves
        // them in flight, phase 5's vmcnt(0) retires them (two conv2 phases of lead)
        uint2 rv[2][4], dv[2][4];
        if constexpr (BWD) {
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const size_t o = ((size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16) * 64 + wc * 32 + m * 16 + 4 * q;
                    rv[m][n] = *(const uint2*)((const char*)A.dy + o * 2);
                    if (A.dot_t) dv[m][n] = *(const uint2*)((const char*)A.dot_t + o * 2);
                    else if (A.gres) dv[m][n] = *(const uint2*)((const char*)A.gres + o * 2);   // 2nd residual
                }
            nhalo += (A.dot_t || A.gres) ? 16 : 8;
        }
        if (k < 2) RSTAMP(10 + k * 14);
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
                if (p == 4) vm_wait(nhalo);              // this phase's taps; the next halo stays in flight
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (!(k + 1 == nmine && p == 5)) issue_taps(P + 1);
            }
            const char* tapp[3] = {ring + (P & 1) * 3 * TAP_BYTES, ring + (P & 1) * 3 * TAP_BYTES + TAP_BYTES,
                                   ring + (P & 1) * 3 * TAP_BYTES + 2 * TAP_BYTES};
            conv2_phase<T>(acc2, a1s, tapp, p - 3, wr, arow2, q, c16);
            if (k < 2) RSTAMP(11 + k * 14 + (p - 3));
        }
        // ---- conv2 epilogue: t_j = acc + b2 (paired-lane 16-B stores), pool partial
        float ps[2][4];
        if constexpr (BWD) {
            // dx = conv1^T(dz1) + dy; DOT: tile sums of dx (as stored) * t_next
#pragma unroll
            for (int m = 0; m < 2; ++m) {
#pragma unroll
                for (int r = 0; r < 4; ++r) ps[m][r] = 0.f;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    acc2[m][n][0] += lo16<T>(rv[m][n].x);
                    acc2[m][n][1] += hi16<T>(rv[m][n].x);
                    acc2[m][n][2] += lo16<T>(rv[m][n].y);
                    acc2[m][n][3] += hi16<T>(rv[m][n].y);
                    if (A.dot_t) {
                        const float tn[4] = {lo16<T>(dv[m][n].x), hi16<T>(dv[m][n].x), lo16<T>(dv[m][n].y),
                                             hi16<T>(dv[m][n].y)};
#pragma unroll
                        for (int r = 0; r < 4; ++r) ps[m][r] += rnd16<T>(acc2[m][n][r]) * tn[r];
                    } else if (A.gres) {                       // a second residual (no DOT)
                        acc2[m][n][0] += lo16<T>(dv[m][n].x);
                        acc2[m][n][1] += hi16<T>(dv[m][n].x);
                        acc2[m][n][2] += lo16<T>(dv[m][n].y);
                        acc2[m][n][3] += hi16<T>(dv[m][n].y);
                    }
                }
            }
        } else {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float4 bb = *(const float4*)(cst + 128 + wc * 32 + m * 16 + 4 * q);
            const float bia[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) ps[m][r] = 0.f;
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc2[m][n][r] += bia[r];
                    ps[m][r] += acc2[m][n][r];
                }
        }
        }
        {
            const bool odd = q & 1;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                uint2 pk[2];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    pk[m].x = pack2<T>(acc2[m][n][0], acc2[m][n][1]);
                    pk[m].y = pack2<T>(acc2[m][n][2], acc2[m][n][3]);
                }
                const uint2 snd = odd ? pk[0] : pk[1];
                uint2 rcv;
                rcv.x = (unsigned)__shfl_xor((int)snd.x, 16, 64);
                rcv.y = (unsigned)__shfl_xor((int)snd.y, 16, 64);
                const uint4 v = odd ? make_uint4(rcv.x, rcv.y, pk[1].x, pk[1].y) : make_uint4(pk[0].x, pk[0].y, rcv.x, rcv.y);
                const size_t px = (size_t)(b * H + h0 + wr * 4 + n) * W + w0 + c16;
                *(uint4*)((char*)d.t + (px * 64 + wc * 32 + (odd ? 16 + 4 * (q - 1) : 4 * q)) * 2) = v;
            }
        }
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float s = group16_sum(ps[m][r]);
                if (c16 == 0) red[wr * 64 + wc * 32 + m * 16 + 4 * q + r] = s;
            }
        // the next halo (DMA + t chunks) landed at the phase-5 wait (vmcnt(0)) in every wave, so
        // the combine below may read other waves' DMA bytes after this barrier; the next tile's
        // first taps (issued at phase 5) and the t stores above stay in flight
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (wave == 0 && d.part)
            d.part[((size_t)b * tpi + tile) * 64 + lane] = (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]);
        if (k < 2) RSTAMP(14 + k * 14);
        // ---- the next tile's x_j: halo image + edge copy + its interior out
        if constexpr (DEFER) {
            if (next) combine_halo(t + nslot, k + 1, tv);
        }
        if constexpr (SEB) {
            if (next) se_halo(t + nslot, k + 1);
        }
        if (k < 2) RSTAMP(15 + k * 14);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef FEN_STAMPS
    RSTAMP(40);
    __syncthreads();
    if (d.stamps && lane < 48 && stamp_lds[wave * 48 + lane] != 0u)
        d.stamps[((size_t)blockIdx.x * 8 + wave) * 48 + lane] = stamp_lds[wave * 48 + lane];
#endif
}

int g_cus = 0;

template <typename T, bool DEFER, bool TRAIN, bool BWD = false, bool GC = false, bool SEB = false>
void launch_rd(const RdArgs& a, int grid, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_rcab_d<T, DEFER, TRAIN, BWD, GC, SEB>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, RD_LDS);
        attr = true;
    }
    hipLaunchKernelGGL((k_rcab_d<T, DEFER, TRAIN, BWD, GC, SEB>), dim3(grid), dim3(512), RD_LDS, s, a);
}

template <typename T>
void launch_rd_t(const fen_rcab_deferred_desc* d, int grid, hipStream_t s) {
    const bool defer = d->tp != nullptr, train = d->z1 != nullptr;
    RdArgs a{};
    a.d = *d;
    if (defer) {
        if (train) launch_rd<T, true, true>(a, grid, s);
        else launch_rd<T, true, false>(a, grid, s);
    } else {
        if (train) launch_rd<T, false, true>(a, grid, s);
        else launch_rd<T, false, false>(a, grid, s);
    }
}

int rd_num_cus() {
    if (g_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus <= 0) g_cus = 256;
    }
    return g_cus;
}

}  // namespace

extern "C" int fen_rcab_deferred_supported(int dtype, int B, int H, int W, int C, int Cr) {
    if ((dtype != FEN_BF16 && dtype != FEN_F16) || C != 64 || Cr <= 0 || Cr > 16 || B <= 0 || H <= 0 || W <= 0 ||
        H % 16 || W % 16)
        return 0;
    if ((size_t)B * H * W * 128 >= (size_t)0x7fff0000) return 0;   // 32-bit buffer offsets
    const size_t ntiles = (size_t)B * (H / 16) * (W / 16);
    return ntiles <= (size_t)MAXG * rd_num_cus() ? 1 : 0;          // gates precomputed per block
}

extern "C" int fen_rcab_deferred(const fen_rcab_deferred_desc* d, void* stream) {
    if (!d || !d->x || !d->w1 || !d->w2 || !d->b1 || !d->b2 || !d->alpha || !d->t || !d->part) return FEN_EINVAL;
    if (!fen_rcab_deferred_supported(d->dtype, d->B, d->H, d->W, d->C, d->Cr)) return FEN_EUNSUPPORTED;
    if (d->tp && (!d->pp || !d->pfc1 || !d->pfc2 || !d->xo)) return FEN_EINVAL;
    if ((d->z1 != nullptr) != (d->a1 != nullptr)) return FEN_EINVAL;
    const int ncu = rd_num_cus();
    const int ntiles = d->B * (d->H / 16) * (d->W / 16);
    const int grid = ntiles < ncu ? ntiles : ncu;
    hipStream_t s = (hipStream_t)stream;
    if (d->dtype == FEN_F16) launch_rd_t<f16>(d, grid, s);
    else launch_rd_t<bf16>(d, grid, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_rcab_bwd_se_supported(int dtype, int B, int H, int W, int C, int Cr) {
    if (!fen_rcab_deferred_supported(dtype, B, H, W, C, Cr)) return 0;
    const int ncu = rd_num_cus();
    const int ntiles = B * (H / 16) * (W / 16);
    const int grid = ntiles < ncu ? ntiles : ncu;
    return (ntiles + grid - 1) / grid <= 6 && (H / 16) * (W / 16) <= 64 ? 1 : 0;
}

extern "C" int fen_rcab_bwd(const fen_rcab_bwd_desc* b, void* stream) {
    if (!b || !b->dt || !b->w2t || !b->w1t || !b->z1 || !b->alpha || !b->dz1 || !b->dalpha_part || !b->dx ||
        !b->dy)
        return FEN_EINVAL;
    if ((b->dot_t != nullptr) != (b->dot_part != nullptr)) return FEN_EINVAL;
    if (b->dres && b->dot_t) return FEN_EINVAL;       // the second residual takes the DOT operand's slot
    const bool seb = b->se_part != nullptr;
    if (seb && (!b->se_s || !b->se_mean || !b->se_hid || !b->se_w1 || !b->se_w2 || !b->se_dw1p || !b->se_dw2p))
        return FEN_EINVAL;
    const int Cr = seb ? b->se_Cr : 16;
    if (!fen_rcab_deferred_supported(b->dtype, b->B, b->H, b->W, b->C, Cr)) return FEN_EUNSUPPORTED;
    // SEB: <= 6 tiles per block (gate rows 4..15 hold their s, g), <= 64 tiles per image
    if (seb && !fen_rcab_bwd_se_supported(b->dtype, b->B, b->H, b->W, b->C, Cr)) return FEN_EUNSUPPORTED;
    const int ncu = rd_num_cus();
    const int ntiles = b->B * (b->H / 16) * (b->W / 16);
    const int grid = ntiles < ncu ? ntiles : ncu;
    RdArgs a{};
    fen_rcab_deferred_desc& d = a.d;
    d.dtype = b->dtype;
    d.B = b->B, d.H = b->H, d.W = b->W, d.C = b->C, d.Cr = Cr;
    d.x = seb ? b->dy : b->dt;                       // SEB: dt is built from dy's halo (and written)
    d.w1 = b->w2t;
    d.w2 = b->w1t;
    d.alpha = b->alpha;
    d.t = b->dx;
    d.part = b->dot_part;
    a.z1 = b->z1;
    a.dz1 = b->dz1;
    a.dpart = b->dalpha_part;
    a.dy = b->dy;
    a.dot_t = b->dot_t;
    a.gres = b->dres;
    if (seb) {
        d.pp = b->se_part;
        d.pfc1 = b->se_w1;
        d.pfc2 = b->se_w2;
        d.res_scale = b->se_res_scale;
        d.inv_hw = 1.0f / (float)(b->H * b->W);
        d.pmean = (float*)b->se_mean;
        d.phid = (float*)b->se_hid;
        d.xo = const_cast<void*>(b->dt);             // (an output in this mode)
        a.se_s = b->se_s;
        a.se_dw1p = b->se_dw1p;
        a.se_dw2p = b->se_dw2p;
    }
    hipStream_t s = (hipStream_t)stream;
    if (seb) {
        if (b->dtype == FEN_F16) launch_rd<f16, false, false, true, false, true>(a, grid, s);
        else launch_rd<bf16, false, false, true, false, true>(a, grid, s);
    } else {
        if (b->dtype == FEN_F16) launch_rd<f16, false, false, true>(a, grid, s);
        else launch_rd<bf16, false, false, true>(a, grid, s);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_rcab_group_end(const fen_rcab_deferred_desc* d, const void* w, const float* bias, const void* res,
                                  void* out, void* stream) {
    if (!d || !d->x || !d->tp || !d->pp || !d->pfc1 || !d->pfc2 || !w || !bias || !res || !out) return FEN_EINVAL;
    if (!fen_rcab_deferred_supported(d->dtype, d->B, d->H, d->W, d->C, d->Cr)) return FEN_EUNSUPPORTED;
    RdArgs a{};
    a.d = *d;
    a.d.w1 = w;
    a.d.w2 = w;
    a.d.b1 = bias;
    a.d.b2 = bias;
    a.d.t = out;
    a.d.part = nullptr;
    a.d.z1 = a.d.a1 = nullptr;
    a.gres = res;
    const int ncu = rd_num_cus();
    const int ntiles = d->B * (d->H / 16) * (d->W / 16);
    const int grid = ntiles < ncu ? ntiles : ncu;
    hipStream_t s = (hipStream_t)stream;
    if (d->dtype == FEN_F16) launch_rd<f16, true, false, false, true>(a, grid, s);
    else launch_rd<bf16, true, false, false, true>(a, grid, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// One ResidualGroup as ONE persistent launch, its activations resident on the CUs
// (reference src/models/blocks.py:161-189: NB x RCAB blocks.py:135-153 with ChannelAttention
// blocks.py:83-92, then the group conv + the group's skip).
//
// Decomposition.  An image of H x 64 pixels is cut into S = H / 8 strips of 8 rows; one
// 512-thread block (one CU: 158 KB of LDS) owns one strip for the whole group, wave w = row w
// of the strip, all 64 channels (64 pixels x 64 channels per wave: 16 accumulator tiles of
// v_mfma_f32_16x16x32_{f16,bf16}).  Between RCABs nothing of the strip leaves the CU:
//   * x_j (the RCAB input) stays in registers in the accumulator layout (32 VGPRs), t_j
//     (conv2's output) in the accumulators themselves; x_{j+1} = x_j + rs * s_j * t_j is
//     computed in registers;
//   * the LDS image (10 rows x 66 columns x 128 B: the strip, one halo row above and below,
//     a zero column each side) holds x_j during conv1 and a1 = PReLU(conv1) during conv2
//     (every conv runs on the strip's own rows only: no halo recompute);
//   * the running conv's 9 filter taps (73.7 KB) are resident in LDS; the next conv's taps
//     stream in by LDS-DMA as the phases free their slots (kh = 1 after the first phase, the
//     rest after the conv).
// What crosses CUs, per RCAB and strip: the SE pool partial (64 floats) and the strip's first
// and last rows of x_j, t_j (the neighbours build their halo rows of x_{j+1} from them) and of
// a1 (the neighbours' conv2 halo rows): <= 48 KB, stored write-through (sc1) and read with
// sc1 loads after the producer's signal -- MI355X_MICROARCH.md, inter-workgroup visibility,
// table row 1: sc1 payload stores -> every storing wave's vmcnt(0) -> barrier -> one lane
// signals; one lane polls with sc1 loads; the polling wave loads after its poll matched, the
// others after a barrier it joins.
//   * the image's strips meet once per RCAB (the gate needs the mean over the whole image):
//     one agent-scope counter per image, +1 per strip and RCAB;
//   * neighbours meet once more inside the RCAB (a1's halo rows): a flag per strip = j + 1.
// Blocks take their strip from a ticket counter in start order, so an image's strips are
// always blocks that are already running: a block only ever waits on running blocks (no
// co-residency assumption; other work on the GPU delays, never deadlocks).  Every wait is
// bounded (the workspace's error word is set instead of hanging).  The last block to finish
// resets the counters for the next launch (graph-replayable).
//
// Precision: 16-bit activations (fp16 / bf16) and weights, fp32 accumulation; x_{j+1}, a1
// and the output rounded to the 16-bit format exactly where the per-launch chain
// (rcab_deferred.hip) rounds them (t rounded before the gate product, as if stored).
#include "strip_common.h"

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace {

using namespace gs;

constexpr int O_IMG = 0;
constexpr int O_FILT = O_IMG + IMG_BYTES;     // 9 tap slots, slot = kh * 3 + kw
constexpr int O_RED = O_FILT + 9 * TAPB;      // [8 waves][64] f32 pool partials
constexpr int O_CST = O_RED + 8 * 64 * 4;     // b1 [64], alpha [64], b2 [64] (group conv: bias in b2)
constexpr int O_GATE = O_CST + 3 * 64 * 4;    // [64] f32: rs * s of the last RCAB
constexpr int O_SCR = O_GATE + 64 * 4;        // mean [64], ticket word
#ifdef FEN_GS_STAMPS
// diagnostic build only (-DFEN_GS_STAMPS, `make gsstamp`, tools/stamp_strip.py): s_memrealtime stamps of waves 0 and 1 in LDS,
// copied to the workspace's tail at the end; no stamp executes in the product build
constexpr int NSTAMP = 100;
constexpr int O_STAMP = O_SCR + 80 * 4;
constexpr int GS_LDS = O_STAMP + 8 * NSTAMP * 2;
#else
constexpr int GS_LDS = O_SCR + 80 * 4;
#endif
static_assert(GS_LDS <= 163840, "LDS budget");
static_assert(O_FILT % 16 == 0 && O_RED % 16 == 0 && O_GATE % 16 == 0, "alignment");


#ifdef FEN_GS_STAMPS
#define GSTAMP(i)                                                                              \
    do {                                                                                       \
        unsigned long long _rt;                                                                \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_rt)::"memory");        \
        if (lane == 0 && (i) < NSTAMP) stamp_lds[wave * NSTAMP + (i)] = (unsigned short)((unsigned)_rt - t_start); \
    } while (0)
#else
#define GSTAMP(i) \
    do {          \
    } while (0)
#endif

// Training (SAVE): a wave's save stores (the backward's operands, 8 buffer stores per row) are
// issued LAST before a wait that only needs the older hand-off traffic (tap DMA, boundary-row
// stores and loads), and that wait leaves them in flight -- s_waitcnt vmcnt(8 per saved row)
// instead of vmcnt(0): vector-memory ops retire in issue order.  A compiler barrier keeps the
// saves behind the older ops.  GS_DRAIN_ALL restores the full drains (A/B).
#ifdef GS_DRAIN_ALL
#define GS_VMCNT_SAVES(n) asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define GS_VMCNT_SAVES(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#endif

// the training saves' cache-policy bits: non-temporal (the backward reads them ~ms later; plain
// stores allocated them in L2 / MALL beside the hand-off rows and filter taps): stage-1 step
// 5.349 / 5.374 / 5.375 vs 5.445 / 5.462 / 5.442 ms (same box)
#ifndef GS_SAVE_AUX
#define GS_SAVE_AUX 2
#endif

// workspace: control words, counters, pool partials, boundary rows
struct Ws {
    size_t cnt, flg, part, bx, bt, ba, bo, stamp, total;
};
__host__ __device__ inline Ws ws_layout(int B, int S) {
    Ws L;
    size_t o = 256;                          // [0] ticket [1] done [2] error [3] launch epoch
    L.cnt = o;
    L.flg = o;  o += (size_t)B * S * 6 * 128;  // per (strip, side, kind) a flag on its own line
    L.part = o; o += (size_t)B * 2 * S * 64 * 8;   // [img][parity][strip][64] {tag, value} granules
    o = (o + 255) & ~(size_t)255;
    const size_t rows = (size_t)B * S * 2 * 2 * ROWB;   // [img][strip][parity][side] rows
    L.bx = o; o += rows;
    L.bt = o; o += rows;
    L.ba = o; o += rows;
    L.bo = o; o += rows / 2;                 // chained groups: a group output's boundary rows [img][strip][side]
    L.stamp = o;
#ifdef FEN_GS_STAMPS
    o += (size_t)B * S * 8 * NSTAMP * 2;            // [block ticket][wave][NSTAMP] u16 (10 ns ticks)
#endif
    L.total = o;
    return L;
}

// chained groups (fen_group_strip_chain): per group its input / output and parameters, in
// device memory after the workspace (a launch's arguments would exceed 4 KB)
struct GsTab {
    const void* x;
    void* y;
    const void* skip;                        // the residual added after the group conv (x; the tail: feat0)
    const void* w[2 * FEN_GS_MAXNB + 1];
    const float* bias[2 * FEN_GS_MAXNB + 1];
    const float* alpha[FEN_GS_MAXNB];
    const float* fc1[FEN_GS_MAXNB];
    const float* fc2[FEN_GS_MAXNB];
    float* s_out[FEN_GS_MAXNB];
    // training (SAVE): the group's saved set, as GsArgs
    void* sv_x[FEN_GS_MAXNB];
    void* sv_z1[FEN_GS_MAXNB];
    void* sv_a1[FEN_GS_MAXNB];
    void* sv_t[FEN_GS_MAXNB];
    float* sv_mean[FEN_GS_MAXNB];
    float* sv_hid[FEN_GS_MAXNB];
    void* x_last;
};
inline size_t gs_tab_offset(int B, int S) { return ((ws_layout(B, S).total + 255) & ~(size_t)255) + 256; }   // rows (header before)
// the table's header (256 B, then the rows): written by prepare, checked by every block of a
// launch before it reads a row -- a workspace that was never prepared (zeros), or prepared for
// other descriptors, fails the check and the launch reports FEN_STATUS_GS_TABLE instead of
// dereferencing a stale or null row
struct GsTabHdr {
    unsigned long long magic;
    unsigned long long hash;                 // FNV-1a of the rows as written
    int rows;
    int pad[59];
};
static_assert(sizeof(GsTabHdr) == 256, "header size");
constexpr unsigned long long GS_TAB_MAGIC = 0x4645'4e43'4841'494eull;   // "FENCHAIN"

struct GsArgs {
    int B, H, S, NB, Cr;
    float res_scale, inv_hw;
    const void* x;                            // group input  [B][H][64][64] NHWC
    void* y;                                  // group output [B][H][64][64]
    const void* w[2 * FEN_GS_MAXNB + 1];      // packed taps: conv1_0, conv2_0, ..., group conv
    const float* bias[2 * FEN_GS_MAXNB + 1];
    const float* alpha[FEN_GS_MAXNB];
    const float* fc1[FEN_GS_MAXNB];           // [Cr][64]
    const float* fc2[FEN_GS_MAXNB];           // [64][Cr]
    float* s_out[FEN_GS_MAXNB];               // optional gates s [B][64] (attention maps)
    char* work;
    int save;                                 // training: the backward's operands out (SAVE)
    void* sv_x[FEN_GS_MAXNB];
    void* sv_z1[FEN_GS_MAXNB];
    void* sv_a1[FEN_GS_MAXNB];
    void* sv_t[FEN_GS_MAXNB];
    float* sv_mean[FEN_GS_MAXNB];
    float* sv_hid[FEN_GS_MAXNB];
    void* x_last;
    int* status;                              // optional: a timed-out wait is reported here
    int fault;                                // test-only: image 0 strip 1 skips one a1 flag
    int pre_elide;                            // training: no z1 save for an RCAB whose slopes are all > 0
    const GsTab* tab;                         // MULTI: ng groups in a row, parameters from here
    unsigned long long tab_hash;              // MULTI: what the header must hold (this launch's rows)
    int ng;
    int tail;                                 // MULTI: + conv_after_body as a group of no RCABs (table row ng)
};

template <typename T, bool SAVE, bool MULTI>
__global__ __launch_bounds__(512, 1) void k_group_strip(const GsArgs A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* img = smem + O_IMG;
    char* filt = smem + O_FILT;
    float* red = (float*)(smem + O_RED);
    float* cst = (float*)(smem + O_CST);
    float* gate = (float*)(smem + O_GATE);
    float* scr = (float*)(smem + O_SCR);
    int* tick_lds = (int*)(scr + 64);
#ifdef FEN_GS_STAMPS
    unsigned short* stamp_lds = (unsigned short*)(smem + O_STAMP);
#endif

    const int tid = threadIdx.x;
    int lane = tid & 63;
    const int wave = wave_id();
    // lane coordinates; re-derived from an opaque copy of the lane id at the top of every
    // chain step, so per-lane addresses are recomputed per step instead of being hoisted out
    // of the chain loop (they would live through the convs, the register peak, and spill)
    int q = lane >> 4, c16 = lane & 15;
#ifdef GS_PRIO
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);   // A/B variant: the SIMDs' younger waves first
#endif
    const int B = A.B, H = A.H, NB = A.NB;
    int S = A.S;
    const Ws L = ws_layout(B, S);
    int* ctl = (int*)A.work;
    // the running group's input / output and parameters: the launch's arguments, or (MULTI,
    // groups g = 0 .. ng-1 in a row, group g's output = group g+1's input) the table's row g
    int g = 0;
    const int NG = MULTI ? A.ng + A.tail : 1;
    // (table entries are wave-uniform: readfirstlane'd, whatever load the compiler picks)
    auto uni = [](const void* p_) -> void* {
        const unsigned long long v = (unsigned long long)p_;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
        return (void*)(((unsigned long long)hi << 32) | lo);
    };
    // the table through the constant address space: scalar loads (it is never written in a launch)
    typedef const __attribute__((address_space(4))) GsTab CTab;
    CTab* ctab = (CTab*)A.tab;
    auto Gx = [&]() -> const void* { return MULTI ? uni(ctab[g].x) : A.x; };
    auto Gy = [&]() -> void* { return MULTI ? uni(ctab[g].y) : A.y; };
    auto Gw = [&](int ci) -> const void* { return MULTI ? uni(ctab[g].w[ci]) : A.w[ci]; };
    auto Gb = [&](int ci) -> const float* { return MULTI ? (const float*)uni(ctab[g].bias[ci]) : A.bias[ci]; };
    auto Ga = [&](int j_) -> const float* { return MULTI ? (const float*)uni(ctab[g].alpha[j_]) : A.alpha[j_]; };

    // ---- the strip: a ticket in start order (an image's strips are running blocks); the
    // launch's epoch (tags of this launch's hand-offs: never equal to an earlier launch's)
    if (tid == 0) {
        tick_lds[0] = __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tick_lds[1] = __hip_atomic_load(ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef FEN_GS_STAMPS
        unsigned long long t0;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
        tick_lds[2] = (int)(unsigned)t0;
        tick_lds[3] = (int)(unsigned)__builtin_amdgcn_s_memtime();
#endif
    }
    // zero the LDS image (halo rows of edge strips and the zero columns stay zero)
    for (int i = tid; i < IMG_BYTES / 16; i += 512) *(uint4*)(img + i * 16) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    if (MULTI) {
        // the table's header against this launch's descriptors (block-uniform: every block reads
        // the same header, so either all blocks run or all leave here, nothing waits on a leaver)
        const GsTabHdr* hdr = (const GsTabHdr*)((const char*)A.tab - sizeof(GsTabHdr));
        const bool bad = hdr->magic != GS_TAB_MAGIC || hdr->hash != A.tab_hash || hdr->rows != A.ng + A.tail;
        if (bad) {
            if (tid == 0) {
                __hip_atomic_fetch_or(ctl + 2, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                strip_finish(ctl, B * S, A.status, FEN_STATUS_GS_FWD);
            }
            return;
        }
    }
    const int ticket = __builtin_amdgcn_readfirstlane(tick_lds[0]);
    const unsigned epoch = (unsigned)__builtin_amdgcn_readfirstlane(tick_lds[1]);
    int kbase = 0, rbase = 0;                               // the group's first step / RCAB (MULTI)
    // a step's tag: unique per (launch, group, step) (MULTI: ng * (nb + 1) < 255 steps)
    auto tag_of = [&](int j) -> unsigned { return (epoch << 8) | (unsigned)(kbase + j + 1); };
#ifdef FEN_GS_STAMPS
    const unsigned t_start = (unsigned)__builtin_amdgcn_readfirstlane(tick_lds[2]);   // the block's clock origin
#endif
    GSTAMP(0);
    int im = ticket / S, strip = ticket - im * S;
    int r0 = strip * SR;
    const bool has_up = strip > 0, has_dn = strip + 1 < S;
    // waves 0 / 7 own the strip's boundary rows (publish them, fetch the neighbours')
    const bool bwave = (wave == 0 && has_up) || (wave == SR - 1 && has_dn);
    const int side = wave == 0 ? 0 : 1;                    // this wave's boundary side
    const int nb_strip = wave == 0 ? strip - 1 : strip + 1;  // the neighbour it reads from
    // x_{j+1}'s halo rows are built by two waves per side (half a row each: 4 of the 8 chunks
    // per lane): waves 0, 2 the upper row, waves 7, 5 the lower one
    const int hs = (wave == 0 || wave == 2) ? 0 : (wave == 5 || wave == SR - 1) ? 1 : -1;
    const bool hwave = hs == 0 ? has_up : hs == 1 ? has_dn : false;
    const int hk0 = (wave == 0 || wave == SR - 1) ? 0 : 4;

    const size_t act_bytes = (size_t)B * H * SW * 128;
    const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc((void*)A.work, 0, (int)L.total, 0x00020000);
    unsigned* flg = (unsigned*)(A.work + L.flg);
    // one flag word per (strip, side, kind), own 128-B line: kind 0 = a1 row, 1 = x / t rows,
    // 2 = a chained group's output row
    auto flag_of = [&](int s_, int sd, int kind) -> unsigned* { return flg + (((im * S + s_) * 2 + sd) * 3 + kind) * 32; };
    auto rowoff = [&](size_t base, int s_, int par, int sd) -> int {
        return (int)(base + ((size_t)((im * S + s_) * 2 + par) * 2 + sd) * ROWB);
    };
    auto booff = [&](int s_, int sd) -> int { return (int)(L.bo + ((size_t)(im * S + s_) * 2 + sd) * ROWB); };

    // ---- filter taps by LDS-DMA: tap k of conv `ci` into slot k (this wave's 1-KB piece)
    auto issue_taps = [&](const void* wp, int k0, int n) {     // taps k0 .. k0 + n - 1
        const i32x4 wr = make_rsrc(wp, 9u * 64u * 128u);
        int ll = lane;
        asm volatile("" : "+v"(ll));
        const int s = wave * 64 + ll, r = s >> 3, pc = s & 7;
        const int v0 = (r * 64 + ((pc ^ ((r >> 1) & 7)) * 8)) * 2;
        for (int k = k0; k < k0 + n; ++k)
            dma16(wr, __builtin_amdgcn_readfirstlane(lds_addr(filt + k * TAPB + wave * 1024)), v0 + k * TAPB);
    };
    auto issue_kh1 = [&](const void* wp) { issue_taps(wp, 3, 3); };
    auto issue_kh02 = [&](const void* wp) {
        issue_taps(wp, 0, 3);
        issue_taps(wp, 6, 3);
    };

    // ---- per-lane helpers on the accumulator layout: lane (q, c16) holds channels
    // 16m + 4q + i (i = 0..3) of pixel 16p + c16 of the wave's row
    uint2 xr[4][4];                                         // x_j, packed 16-bit
    auto px_off = [&](int row, int p) -> size_t {           // byte offset of (image row, pixel 16p + c16)
        return ((size_t)(im * H + row) * SW + 16 * p + c16) * 128;
    };
    auto write_row_lds = [&](int lrow, const uint2 (&v)[4][4]) {
        int qq = q, cc = c16;
        asm volatile("" : "+v"(qq), "+v"(cc));              // addresses per use, not hoisted
        const int key = (cc + 1) & 7;
        char* rb = img + lrow * IROW + (cc + 1) * 128 + (qq & 1) * 8;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            char* mb = rb + (((2 * m + (qq >> 1)) ^ key) << 4);
#pragma unroll
            for (int p = 0; p < 4; ++p) *(uint2*)(mb + p * 2048) = v[m][p];
        }
    };
    // a strip row (accumulator layout) out as 16-B chunks through `rs` at byte offset `base`
    auto store_row = [&](__amdgpu_buffer_rsrc_t rs, int base, const uint2 (&v)[4][4], int aux) {
        int qq = q, cc = c16;
        asm volatile("" : "+v"(qq), "+v"(cc));
        const int lb = base + cc * 128 + chunk_of(0, qq) * 16;
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int mp = 0; mp < 2; ++mp) {
                const uint4 u = pair16(v[2 * mp][p], v[2 * mp + 1][p]);
                const int off = lb + p * 2048 + mp * 64;
                if (aux == 16) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, u), rs, off, 0, 16);
                else if (aux == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, u), rs, off, 0, 2);
                else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, u), rs, off, 0, 0);
            }
    };
    // training: the wave's row of a saved activation (the backward reads it ~ms later), stored
    // non-temporal (GS_SAVE_AUX)
    auto save_row = [&](void* base, const uint2 (&v)[4][4]) {
        void* bp = base;
        asm volatile("" : "+s"(bp));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(bp, 0, (int)act_bytes, 0x00020000);
        store_row(rs, (int)((size_t)(im * H + r0 + wave) * SW * 128), v, GS_SAVE_AUX);
    };
    // a boundary row (16-B chunks, lane handles chunks lane + 64 k) -> LDS image row lrow
    auto halo_to_lds = [&](int lrow, const uint4 (&v)[8]) {
        int ll = lane;
        asm volatile("" : "+v"(ll));
        char* hb = img + lrow * IROW + hcol((ll >> 3) + 1, ll & 7);   // pixel + 8 k keeps the key
#pragma unroll
        for (int k = 0; k < 8; ++k) *(uint4*)(hb + k * 1024) = v[k];
    };
    auto load_row = [&](int off, uint4 (&v)[8]) {           // sc1: a handed-off row
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wsr, off + (lane + 64 * k) * 16, 0, 16));
    };

    // ================= start-up: conv1_0's taps, x_0, constants =================
    issue_taps(Gw(0), 0, 9);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)Gx(), 0, (int)act_bytes, 0x00020000);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int p = 0; p < 4; ++p)
            xr[m][p] = *(const uint2*)((const char*)Gx() + px_off(r0 + wave, p) + (16 * m + 4 * q) * 2);
    if (bwave) {
        uint4 hv[8];
        const int row = wave == 0 ? r0 - 1 : r0 + SR;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = lane + 64 * k;
            hv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xrs, (int)(((size_t)(im * H + row) * SW) * 128) + i * 16, 0, 0));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        halo_to_lds(wave == 0 ? 0 : SR + 1, hv);
    }
    float cv = 0.f;
    if (wave == 2) cv = Gb(0)[lane];
    if (wave == 3) cv = Ga(0)[lane];
    if (wave == 4) cv = Gb(1)[lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave >= 2 && wave <= 4) cst[(wave - 2) * 64 + lane] = cv;
    write_row_lds(wave + 1, xr);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();                                        // conv1_0's taps (every wave's pieces) landed
    GSTAMP(1);

    // ================= the chain: RCAB j = 0 .. NB-1, then the group conv =================
    // Per RCAB, five barriers: B_X (conv1's image complete), B_E (conv1 done), B_Y (a1 image
    // complete), B_Z (the strip's pool partial complete), B_G (the gate known).  Phase 1 of each
    // conv reads the wave's own row only and runs without a barrier.  The gate's pool partial
    // is computed from a1 before conv2's phases 2-3 (the conv is linear: sum over the strip's
    // pixels of conv2(a1) = W2 applied to a1's per-channel sums, less the columns / rows a tap
    // reads past the image's edge), so the image's strips exchange it while conv2 still runs.
    uint2 tr[4][4];                                         // t_j as stored (16-bit), for the next combine
    const int khP2 = wave == 0 ? 2 : 0, khP3 = 2 - khP2;   // wave 0's upper halo row is read last
    bool ok = true;
    for (;;) {                                              // groups (one unless MULTI)
    kbase = g * (NB + 1), rbase = g * NB;
    const bool gtail = MULTI && g >= A.ng;                  // conv_after_body: a "group" of no RCABs
    for (int j = 0;; ++j) {                                // one exit: the group conv's break
        const bool gc = j == (gtail ? 0 : NB);
        // boundary rows and pool partials double-buffered by RCAB count (not step: a group conv
        // publishes neither, and each buffer's reuse is ordered by the hand-offs of the RCAB between)
        const int par = (rbase + j) & 1;
        const int sb = 2 + 9 * j;                           // this step's stamp slots
        {
            // opaque per step: what is computed from these is recomputed here, not hoisted
            int ll = lane;
            asm volatile("" : "+v"(ll), "+s"(im), "+s"(strip), "+s"(S), "+s"(r0));
            lane = ll, q = ll >> 4, c16 = ll & 15;
        }
        const int ci = gc ? (gtail ? 0 : 2 * NB) : 2 * j;
        GSTAMP(sb);
        uint4 nx[4], nt[4];
        // the halo waves poll the neighbour's flag before issuing their tap DMA: a poll waits on
        // every older vector-memory op of its wave (vmcnt(0))
#ifndef GS_OLD_ORDER
        const bool dma_late = hwave;
#else
        const bool dma_late = false;
#endif
        if (j > 0 || g > 0) {
            if (!dma_late) issue_kh02(Gw(ci));              // this conv's kh = 0, 2 taps (slots free since B_G)
            if (wave >= 2 && wave <= 4) cst[(wave - 2) * 64 + lane] = cv;   // read after B_E / B_Z
        }
        if (j > 0) {
            // ---- x_j = x_{j-1} + rs * s * t_{j-1} (t as stored: rounded), own row in registers
            float gt[4][4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float4 gv = *(const float4*)(gate + 16 * m + 4 * q);
                gt[m][0] = gv.x, gt[m][1] = gv.y, gt[m][2] = gv.z, gt[m][3] = gv.w;
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    __builtin_amdgcn_sched_barrier(0);
                    const float x0 = lo16<T>(xr[m][p].x), x1 = hi16<T>(xr[m][p].x);
                    const float x2 = lo16<T>(xr[m][p].y), x3 = hi16<T>(xr[m][p].y);
                    xr[m][p] = pk4<T>(lo16<T>(tr[m][p].x) * gt[m][0] + x0, hi16<T>(tr[m][p].x) * gt[m][1] + x1,
                                      lo16<T>(tr[m][p].y) * gt[m][2] + x2, hi16<T>(tr[m][p].y) * gt[m][3] + x3);
                }
        }
        if (j > 0 || g > 0) write_row_lds(wave + 1, xr);    // (a chained group's x_0: the previous output)
        // x_j's boundary rows for the neighbours (their halo rows of x_{j+1})
        if (!gc && bwave) store_row(wsr, rowoff(L.bx, strip, par, side), xr, 16);
        if (j > 0 && hwave) {
            // the neighbour's x_{j-1}, t_{j-1} rows (this wave's half), after its flag (its
            // storing wave drained them, then signalled): this wave polls and loads (row 1);
            // the loads land during phase 1
            const int pp = (rbase + j - 1) & 1;
            const int ns = hs == 0 ? strip - 1 : strip + 1;
            ok = ok && poll_eq(flag_of(ns, 1 - hs, 1), tag_of(j - 1));
            const int ox = rowoff(L.bx, ns, pp, 1 - hs) + (lane + 64 * hk0) * 16;
            const int ot = rowoff(L.bt, ns, pp, 1 - hs) + (lane + 64 * hk0) * 16;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                nx[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wsr, ox + k * 1024, 0, 16));
                nt[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wsr, ot + k * 1024, 0, 16));
            }
        }
        if (MULTI && j == 0 && g > 0 && hwave) {
            // a chained group's x_0 halo: this wave's half of the neighbour's previous group
            // output row, after its flag (kind 2)
            const int ns = hs == 0 ? strip - 1 : strip + 1;
            ok = ok && poll_eq(flag_of(ns, 1 - hs, 2), tag_of(-1));
            const int ox = booff(ns, 1 - hs) + (lane + 64 * hk0) * 16;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                nx[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wsr, ox + k * 1024, 0, 16));
        }
        if (dma_late && (j > 0 || g > 0)) issue_kh02(Gw(ci));
        if (SAVE && j > 0) {                                // x_0 is the group input
            asm volatile("" ::: "memory");                  // the saves after every op the wait below needs
            save_row(MULTI ? uni(gc ? ctab[g].x_last : ctab[g].sv_x[j]) : gc ? A.x_last : A.sv_x[j], xr);
        }

        // ================= conv1 (or the group conv): 3 phases =================
        f32x4 acc[4][4];                                    // conv1 (group conv), then conv2
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[m][p] = zero4();
        // phase 1 (kh = 1) reads the wave's own row only: no barrier.  Its taps are visible since
        // B_G (or the start-up barrier); a wave whose combine is short starts its MFMAs while its
        // SIMD partner still builds halo rows
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GSTAMP(sb + 1);
        conv_phase<T>(acc, img, filt, 1, wave, q, c16);
        GSTAMP(sb + 2);
        if (SAVE && j > 0) GS_VMCNT_SAVES(8);                 // this conv's taps; the halo rows (x_j's save in flight)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (j > 0 && hwave) {                               // its half of x_j's halo row, same arithmetic
            const float4 ga = *(const float4*)(gate + (lane & 7) * 8);
            const float4 gb = *(const float4*)(gate + (lane & 7) * 8 + 4);
            const float g8[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
            char* hb = img + (hs == 0 ? 0 : SR + 1) * IROW + hcol((lane >> 3) + 1, lane & 7) + hk0 * 1024;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float xf[8], tf[8], yv[8];
                unpack16<T>(nx[k], xf);
                unpack16<T>(nt[k], tf);
#pragma unroll
                for (int e = 0; e < 8; ++e) yv[e] = tf[e] * g8[e] + xf[e];
                *(uint4*)(hb + k * 1024) = pack16<T>(yv);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (MULTI && j == 0 && g > 0 && hwave) {
            char* hb = img + (hs == 0 ? 0 : SR + 1) * IROW + hcol((lane >> 3) + 1, lane & 7) + hk0 * 1024;
#pragma unroll
            for (int k = 0; k < 4; ++k) *(uint4*)(hb + k * 1024) = nx[k];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __syncthreads();                                    // B_X: every image row written; kh = 1 slots free
        if (!gc) issue_kh1(Gw(ci + 1));
        else if (MULTI && g + 1 < NG) issue_kh1(uni(ctab[g + 1].w[0]));   // the next group's conv1_0
        uint2 x0r[4][4];                                    // the group conv's skip input, own row
        if (MULTI && gc) {
            // issued here, in flight under phases 2-3 (the chained kernel has the registers);
            // sc1 loads: a chained group's input is the previous group's output, rows this wave
            // stored in this launch
            const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(uni(ctab[g].skip), 0, (int)act_bytes, 0x00020000);
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    x0r[m][p] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                              grs, (int)(px_off(r0 + wave, p) + (16 * m + 4 * q) * 2), 0, 16));
        }
        conv_phase<T>(acc, img, filt, khP2, wave, q, c16);
        conv_phase<T>(acc, img, filt, khP3, wave, q, c16);
        GSTAMP(sb + 3);
        if (gc) {
            // ---- out = conv + bias + the group input (blocks.py:188-189): its own rows read
            // again here (once per launch; kept out of the conv's register peak)
            if (!MULTI) {
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int p = 0; p < 4; ++p)
                        x0r[m][p] = *(const uint2*)((const char*)A.x + px_off(r0 + wave, p) + (16 * m + 4 * q) * 2);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint2 ov[4][4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float4 bb = *(const float4*)(cst + 128 + 16 * m + 4 * q);
                const float bia[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    float v[4];
                    v[0] = acc[m][p][0] + bia[0] + lo16<T>(x0r[m][p].x);
                    v[1] = acc[m][p][1] + bia[1] + hi16<T>(x0r[m][p].x);
                    v[2] = acc[m][p][2] + bia[2] + lo16<T>(x0r[m][p].y);
                    v[3] = acc[m][p][3] + bia[3] + hi16<T>(x0r[m][p].y);
                    ov[m][p] = pk4<T>(v[0], v[1], v[2], v[3]);
                }
            }
            const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(Gy(), 0, (int)act_bytes, 0x00020000);
            const bool handoff = MULTI && g + 1 < NG;
            if (handoff && wave >= 2 && wave <= 4) {
                // the next group's first constants: its first RCAB's b1, alpha, b2, or the tail
                // conv's bias (the group conv's slot); issued before the stores (see below)
                CTab& nt_ = ctab[g + 1];
                if (g + 1 < A.ng) cv = ((const float*)uni(wave == 2 ? nt_.bias[0] : wave == 3 ? nt_.alpha[0] : nt_.bias[1]))[lane];
                else cv = wave == 4 ? ((const float*)uni(nt_.bias[0]))[lane] : 0.f;
            }
            // the boundary rows for the neighbours before the output row: the flag waits for
            // those (and every older op) only, the output's 8 stores stay in flight
            if (handoff && bwave) store_row(wsr, booff(strip, side), ov, 16);
            store_row(yrs, (int)((size_t)(im * H + r0 + wave) * SW * 128), ov, 0);
            if (MULTI) {
                // the next group: x_0 = this output (registers), its boundary rows to the
                // neighbours (kind 2), its first RCAB's constants.  x and t are reassigned on
                // every path out of the step (t is dead until the next conv2: a constant ends the
                // last t's live range at this step's combine instead of holding it through the
                // group conv)
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        xr[m][p] = ov[m][p];
                        tr[m][p] = make_uint2(0u, 0u);
                    }
                if (handoff) {
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    if (bwave && lane == 0)
                        __hip_atomic_store(flag_of(strip, side, 2), tag_of(NB), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __syncthreads();                        // the group conv's image reads done; the next conv1's kh = 1 taps visible
                }
            }
            break;
        }
        // ---- conv1 epilogue: a1 = PReLU(conv1 + b1) -> LDS (own row), boundary rows out; the
        // row's per-channel sums of a1 (fp32, before the 16-bit rounding conv2 reads) -> red[wave].
        // It runs BEFORE the barrier B_E (only the LDS write of the a1 row must wait for every
        // wave's conv1 reads of x_j): a wave that finished its phases early computes its epilogue
        // while its SIMD partner still issues MFMAs, instead of idling at B_E (GS_LATE_EPI: after)
        uint2 av[4][4];
        auto a1_epilogue = [&]() {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float4 bb = *(const float4*)(cst + 16 * m + 4 * q);
                const float4 aa = *(const float4*)(cst + 64 + 16 * m + 4 * q);
                const float bia[4] = {bb.x, bb.y, bb.z, bb.w}, alp[4] = {aa.x, aa.y, aa.z, aa.w};
                float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    float v[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = prelu_f(acc[m][p][i] + bia[i], alp[i]);
                    av[m][p] = pk4<T>(v[0], v[1], v[2], v[3]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) rs[i] += v[i];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float s = group16_sum(rs[i]);
                    if (c16 == 0) red[wave * 64 + 16 * m + 4 * q + i] = s;
                }
            }
        };
#ifndef GS_LATE_EPI
        constexpr bool early = true;
#else
        constexpr bool early = false;
#endif
        if (early) a1_epilogue();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // this wave's pieces of conv2's kh = 1 taps
        __syncthreads();                                    // B_E: x_j's reads done (all slots free); those taps visible
        issue_kh02(Gw(ci + 1));
        uint2 zv[4][4];
        // pre_elide: z1 is recoverable from a1 when all 64 slopes of RCAB j are > 0 (lane = channel)
        const bool wz1 = SAVE && !(A.pre_elide && __ballot(cst[64 + lane] > 0.f) == ~0ull);
        if (SAVE) {                                         // z1 = conv1 + b1 (PReLU's input)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float4 bb = *(const float4*)(cst + 16 * m + 4 * q);
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    zv[m][p] = pk4<T>(acc[m][p][0] + bb.x, acc[m][p][1] + bb.y, acc[m][p][2] + bb.z, acc[m][p][3] + bb.w);
            }
        }
        if (!early) a1_epilogue();
        write_row_lds(wave + 1, av);
        if (bwave) store_row(wsr, rowoff(L.ba, strip, par, side), av, 16);
        if (SAVE) {
            asm volatile("" ::: "memory");
            if (wz1) save_row(MULTI ? uni(ctab[g].sv_z1[j]) : A.sv_z1[j], zv);
            save_row(MULTI ? uni(ctab[g].sv_a1[j]) : A.sv_a1[j], av);
        }
        // ================= conv2 =================
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[m][p] = zero4();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GSTAMP(sb + 4);
        conv_phase<T>(acc, img, filt, 1, wave, q, c16);     // own a1 row only: no barrier
        GSTAMP(sb + 5);
        if (SAVE && wz1) GS_VMCNT_SAVES(16);                  // conv2's other taps; the a1 boundary stores
        else if (SAVE) GS_VMCNT_SAVES(8);                     // (a1's save only)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // a1's boundary row is out: its storing wave signals for itself (one lane, after its drain)
        if (bwave && lane == 0 && !(A.fault && ticket == 1 && j == 0 && side == 0))
            __hip_atomic_store(flag_of(strip, side, 0), tag_of(j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();                                    // B_Y: a1 image and row sums complete; conv2's taps visible
        // ---- the strip's pool partial of t_j (blocks.py:89 AdaptiveAvgPool of conv2's output,
        // less the bias): sum over the strip's output pixels of conv2(a1) = sum_{ci, tap}
        // W2[tap][co][ci] * u[ci][tap], u = the sum of a1[ci] over the input pixels the tap reads
        // -- the strip's a1 sum, less column 0 (kw = 2) / column W-1 (kw = 0), less the image's
        // row 0 (kh = 2; strip 0's first row) / row H-1 (kh = 0; the last strip's last row),
        // whose inputs lie past the image's edge.  Slice sl takes channels ci = 8 sl .. 8 sl + 7:
        // lane (r, c) reads row r's sums of channel 8 sl + c and both edge pixels (from the LDS
        // image), the sums over the 8 rows by lane exchanges; then lane co accumulates
        // W2[tap][co][8 sl .. 8 sl + 7] * u (fixed order) into red, in the slots only this slice
        // reads (a permutation: co -> [co >> 3][8 sl + (co & 7)]).
        auto pool_slice = [&](int sl) {
            int ll = lane;
            asm volatile("" : "+v"(ll));
            const int r = ll >> 3, c = ll & 7, cw = 8 * sl + c;
            const float rsum = red[r * 64 + cw];
            const char* rb = img + (r + 1) * IROW + 2 * c;
            const float p0 = lo16<T>((unsigned)*(const unsigned short*)(rb + hcol(1, sl)));
            const float pl = lo16<T>((unsigned)*(const unsigned short*)(rb + hcol(SW, sl)));
            // every lane of channel c: the strip's sums less column W-1 (kw = 0), -, less column 0 (kw = 2)
            const float tt = sum_lanes_x8(rsum), c0 = sum_lanes_x8(p0), cl = sum_lanes_x8(pl);
            const float bs[3] = {tt - cl, tt, tt - c0};
            // lane co: sum_c sum_kw bs[kw](c) * sum_kh W2[kh][kw][co][8 sl + c]; bs of channel c from
            // lane c of the lane's row of 16 (row_newbcast)
            const char* wb = filt + ll * 128 + ((sl ^ ((ll >> 1) & 7)) << 4);
            float P = 0.f;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                float w0[8], w1[8], w2[8];
                unpack16<T>(*(const uint4*)(wb + kw * TAPB), w0);
                unpack16<T>(*(const uint4*)(wb + (3 + kw) * TAPB), w1);
                unpack16<T>(*(const uint4*)(wb + (6 + kw) * TAPB), w2);
                float ws[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) ws[e] = w0[e] + w1[e] + w2[e];
                bcast8_fma(P, bs[kw], ws);
            }
            if (strip == 0 || strip == S - 1) {
                // the image's first / last row: the taps that read past the top (kh = 2) / bottom
                // (kh = 0) edge drop that row's terms.  Row 0's sums sit in lanes 0..7, row 7's in 56..63
                const float ev[3] = {rsum - pl, rsum, rsum - p0};
#pragma unroll
                for (int side_ = 0; side_ < 2; ++side_) {
                    if (side_ == 0 ? strip != 0 : strip != S - 1) continue;
                    const int kh = side_ == 0 ? 2 : 0, l0 = side_ == 0 ? 0 : 56;
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        float wk[8];
                        unpack16<T>(*(const uint4*)(wb + (3 * kh + kw) * TAPB), wk);
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            P -= wk[e] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ev[kw]), l0 + e));
                    }
                }
            }
            red[(ll >> 3) * 64 + 8 * sl + (ll & 7)] = P;
        };
        // the strip's partial as {tag, value} granules (one 8-B sc1 store each), slices in order
        auto publish_partial = [&]() {
            float s_ = 0.f;
#pragma unroll
            for (int w = 0; w < SR; ++w) s_ += red[(lane >> 3) * 64 + 8 * w + (lane & 7)];
            unsigned long long* pg = (unsigned long long*)(A.work + L.part) + ((size_t)(im * 2 + par) * S + strip) * 64 + lane;
            __hip_atomic_store(pg, ((unsigned long long)tag_of(j) << 32) | __float_as_uint(s_), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        };
        pool_slice(wave);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();                                    // B_Z: the partial's eight channel slices in red; kh = 1 slots free
        issue_kh1(Gw(j + 1 < NB ? ci + 2 : 2 * NB));
        if (wave == 3) publish_partial();
        GSTAMP(sb + 6);
        conv_phase<T>(acc, img, filt, khP2, wave, q, c16);
        if (bwave) {
            // the neighbour's a1 row -> this wave's private halo row (only this wave reads it)
            ok = ok && poll_eq(flag_of(nb_strip, 1 - side, 0), tag_of(j));
            uint4 hv[8];
            load_row(rowoff(L.ba, nb_strip, par, 1 - side), hv);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            halo_to_lds(wave == 0 ? 0 : SR + 1, hv);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        conv_phase<T>(acc, img, filt, khP3, wave, q, c16);
        GSTAMP(sb + 7);
        // ---- conv2 epilogue: t_j = conv2 + b2 as stored (rounded), kept for the next combine
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 bb = *(const float4*)(cst + 128 + 16 * m + 4 * q);
#pragma unroll
            for (int p = 0; p < 4; ++p)
                tr[m][p] = pk4<T>(acc[m][p][0] + bb.x, acc[m][p][1] + bb.y, acc[m][p][2] + bb.z, acc[m][p][3] + bb.w);
        }
        if (bwave) store_row(wsr, rowoff(L.bt, strip, par, side), tr, 16);   // t_j's boundary row
        if (wave == 1) {
            // the gate of RCAB j (blocks.py:83-92): mean over the image from the S strip
            // partials, each an 8-B {tag, value} granule (the data is the flag: sc1 loads
            // swept until every tag is this RCAB's), summed in strip order, + b2; FC1 -> ReLU
            // -> FC2 -> sigmoid.  FC1 rows jj >= Cr read past fc1's end: 0, so hid_jj = 0 and
            // FC2's columns k >= Cr (finite values of the next rows, or 0 past the end) drop out
            // (the weight pointers made opaque here: buffer loads are speculatable, and
            // hoisted out of this wave's branch they held 32 VGPRs in every wave)
            const int Cr = A.Cr, jj = lane & 15, qq = lane >> 4;
            const float* f1p = MULTI ? (const float*)uni(ctab[g].fc1[j]) : A.fc1[j];
            const float* f2p = MULTI ? (const float*)uni(ctab[g].fc2[j]) : A.fc2[j];
            const float* b2p = Gb(2 * j + 1);
            asm volatile("" : "+s"(f1p), "+s"(f2p), "+s"(b2p));
            const __amdgpu_buffer_rsrc_t f1r = __builtin_amdgcn_make_buffer_rsrc((void*)f1p, 0, Cr * 64 * 4, 0x00020000);
            const __amdgpu_buffer_rsrc_t f2r = __builtin_amdgcn_make_buffer_rsrc((void*)f2p, 0, Cr * 64 * 4, 0x00020000);
            float w1v[16], w2v[16];
#pragma unroll
            for (int k4 = 0; k4 < 16; k4 += 4) {
                const float4 a = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                f1r, (jj * 64 + 16 * qq + k4) * 4, 0, 0));
                w1v[k4] = a.x, w1v[k4 + 1] = a.y, w1v[k4 + 2] = a.z, w1v[k4 + 3] = a.w;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k)
                w2v[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(f2r, (lane * Cr + k) * 4, 0, 0));
            const float b2v = b2p[lane];
            const unsigned tg = tag_of(j);
            const unsigned long long* pg =
                (const unsigned long long*)(A.work + L.part) + ((size_t)(im * 2 + par) * S) * 64 + lane;
            // every granule load in flight at once, no branch per strip: strips past S re-read
            // strip 0 and drop out of the sum and the check
            float msum = 0.f;
            bool got = false;
            for (int it = 0; it < SPIN_MAX && ok; ++it) {
                unsigned long long gv[16];
#pragma unroll
                for (int s_ = 0; s_ < 16; ++s_)
                    gv[s_] = __hip_atomic_load(pg + (s_ < S ? s_ : 0) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                unsigned bad = 0u;
                float ms = 0.f;                             // in strip order
#pragma unroll
                for (int s_ = 0; s_ < 16; ++s_) {
                    const bool in = s_ < S;
                    ms += in ? __uint_as_float((unsigned)gv[s_]) : 0.f;
                    bad |= (unsigned)(in & ((unsigned)(gv[s_] >> 32) != tg));
                }
                msum = ms;
                if (__all(bad == 0u)) {
                    got = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            ok = ok && got;
            const float mean = msum * A.inv_hw + b2v;
            scr[lane] = mean;
            float h = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) h += w1v[k] * scr[16 * qq + k];
            h += __shfl_xor(h, 16, 64);
            h += __shfl_xor(h, 32, 64);
            const float hid = fmaxf(h, 0.f);
            float z = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) z += w2v[k] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hid), k));
            const float sg = 1.f / (1.f + expf(-z));
            gate[lane] = sg * A.res_scale;
            float* so = MULTI ? (float*)uni(ctab[g].s_out[j]) : A.s_out[j];
            if (strip == 0 && so) so[im * 64 + lane] = sg;
            if (strip == 0 && SAVE) {
                float* smn = MULTI ? (float*)uni(ctab[g].sv_mean[j]) : A.sv_mean[j];
                float* shd = MULTI ? (float*)uni(ctab[g].sv_hid[j]) : A.sv_hid[j];
                smn[im * 64 + lane] = mean;
                if (lane < Cr) shd[im * Cr + lane] = hid;
            }
        }
        if (wave >= 2 && wave <= 4) {                       // the next conv's epilogue constants
            const bool ng = j + 1 == NB;
            const float* src = ng ? (wave == 4 ? Gb(2 * NB) : nullptr)
                                  : (wave == 2 ? Gb(2 * j + 2) : wave == 3 ? Ga(j + 1) : Gb(2 * j + 3));
            cv = src ? src[lane] : 0.f;
        }
        // x_j's and t_j's boundary rows out: drained, then the storing wave signals for itself
        if (SAVE) {                                         // t_j's save: last, left in flight
            asm volatile("" ::: "memory");
            save_row(MULTI ? uni(ctab[g].sv_t[j]) : A.sv_t[j], tr);
            GS_VMCNT_SAVES(8);
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (bwave && lane == 0) __hip_atomic_store(flag_of(strip, side, 1), tag_of(j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GSTAMP(sb + 8);
        __syncthreads();                                    // B_G: the gate in LDS; conv2's reads done (all slots free)
    }
    if (!MULTI || ++g >= NG) break;
    }
    GSTAMP(NSTAMP - 1);
    // ---- the last block out advances the epoch and resets the ticket counters for the next launch
    if (!ok) __hip_atomic_fetch_or(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) strip_finish(ctl, B * S, A.status, FEN_STATUS_GS_FWD);
#ifdef FEN_GS_STAMPS
    __syncthreads();
    // the block's shader clock: s_memtime cycles / 16 over the block's life, in wave 1's end
    // slot (the tools read the end stamp of wave 0 only)
    if (tid == 0)
        stamp_lds[NSTAMP + NSTAMP - 1] = (unsigned short)(((unsigned)__builtin_amdgcn_s_memtime() - (unsigned)tick_lds[3]) >> 4);
    __syncthreads();
    {
        unsigned short* dst = (unsigned short*)(A.work + L.stamp) + (size_t)ticket * 8 * NSTAMP;
        for (int i = tid; i < 8 * NSTAMP; i += 512) dst[i] = stamp_lds[i];
    }
#endif
}

int g_gs_cus = 0;
int gs_num_cus() {
    if (g_gs_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_gs_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_gs_cus <= 0) g_gs_cus = 256;
    }
    return g_gs_cus;
}

template <typename T, bool SAVE, bool MULTI = false>
void launch_gs(const GsArgs& a, int grid, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_group_strip<T, SAVE, MULTI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  GS_LDS);
        attr = true;
    }
    hipLaunchKernelGGL((k_group_strip<T, SAVE, MULTI>), dim3(grid), dim3(512), GS_LDS, s, a);
}

// FNV-1a over the table rows: the launch recomputes it from its own descriptors and the kernel
// compares it with the header prepare wrote
unsigned long long tab_hash(const std::vector<GsTab>& tab) {
    unsigned long long h = 0xcbf29ce484222325ull;
    const unsigned char* p = (const unsigned char*)tab.data();
    for (size_t i = 0, n = tab.size() * sizeof(GsTab); i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

// the table goes to the device as kernel arguments (no host buffer outlives the call, no host
// sync, capturable): 3.5-KB chunks, one tiny launch each
struct TabChunk {
    unsigned int w[896];
};
__global__ __launch_bounds__(256) void k_tab_write(unsigned int* __restrict__ dst, const TabChunk c, int nw) {
    for (int i = threadIdx.x; i < nw; i += 256) dst[i] = c.w[i];
}

int chain_tab(const fen_group_strip_desc* d, int ng, const fen_group_strip_chain_tail* tail, std::vector<GsTab>& tab) {
    if (!d || ng <= 0) return FEN_EINVAL;
    const fen_group_strip_desc& d0 = d[0];
    if (!fen_group_strip_supported(d0.dtype, d0.B, d0.H, d0.W, d0.C, d0.Cr, d0.nb)) return FEN_EUNSUPPORTED;
    const int rows = ng + (tail ? 1 : 0);
    if (rows * (d0.nb + 1) > 254) return FEN_EUNSUPPORTED;                    // step tags
    tab.assign(rows, GsTab{});
    for (int g = 0; g < ng; ++g) {
        const fen_group_strip_desc& e = d[g];
        if (e.dtype != d0.dtype || e.B != d0.B || e.H != d0.H || e.W != d0.W || e.C != d0.C || e.Cr != d0.Cr ||
            e.nb != d0.nb || e.res_scale != d0.res_scale || (e.save != 0) != (d0.save != 0) || e.work != d0.work ||
            e.pre_elide != d0.pre_elide)
            return FEN_EINVAL;
        if (!e.x || !e.y || !e.wg || !e.bg || e.x == e.y) return FEN_EINVAL;
        if (g > 0 && e.x != d[g - 1].y) return FEN_EINVAL;                   // a chain: output -> next input
        GsTab& t = tab[g];
        t.x = e.x, t.y = e.y, t.skip = e.x;
        for (int j = 0; j < e.nb; ++j) {
            if (!e.w1[j] || !e.b1[j] || !e.alpha[j] || !e.w2[j] || !e.b2[j] || !e.fc1[j] || !e.fc2[j])
                return FEN_EINVAL;
            t.w[2 * j] = e.w1[j], t.bias[2 * j] = e.b1[j];
            t.w[2 * j + 1] = e.w2[j], t.bias[2 * j + 1] = e.b2[j];
            t.alpha[j] = e.alpha[j], t.fc1[j] = e.fc1[j], t.fc2[j] = e.fc2[j], t.s_out[j] = e.s_out[j];
        }
        t.w[2 * e.nb] = e.wg, t.bias[2 * e.nb] = e.bg;
        if (e.save) {                                    // as fen_group_strip's checks
            if (!e.x_last) return FEN_EINVAL;
            t.x_last = e.x_last;
            for (int j = 0; j < e.nb; ++j) {
                if ((j > 0 && !e.sv_x[j]) || !e.sv_z1[j] || !e.sv_a1[j] || !e.sv_t[j] || !e.sv_mean[j] ||
                    !e.sv_hid[j] || !e.s_out[j])
                    return FEN_EINVAL;
                t.sv_x[j] = e.sv_x[j], t.sv_z1[j] = e.sv_z1[j], t.sv_a1[j] = e.sv_a1[j], t.sv_t[j] = e.sv_t[j];
                t.sv_mean[j] = e.sv_mean[j], t.sv_hid[j] = e.sv_hid[j];
            }
        }
    }
    if (tail) {
        // conv_after_body (custom.py:172-175): y = conv(body output) + bias + skip
        if (!tail->w || !tail->bias || !tail->skip || !tail->y || tail->y == d[ng - 1].y || tail->y == tail->skip)
            return FEN_EINVAL;
        GsTab& t = tab[ng];
        t.x = d[ng - 1].y, t.y = tail->y, t.skip = tail->skip;
        t.w[0] = tail->w, t.bias[0] = tail->bias;
        if (d0.save) t.x_last = d[ng - 1].y;                     // (unused: no save in a group of no RCABs)
    }
    if (!d0.work || d0.work_bytes < gs_tab_offset(d0.B, d0.H / SR) + (size_t)rows * sizeof(GsTab)) return FEN_EINVAL;
    return FEN_OK;
}

}  // namespace

extern "C" int fen_group_strip_supported(int dtype, int B, int H, int W, int C, int Cr, int nb) {
    if ((dtype != FEN_BF16 && dtype != FEN_F16) || C != 64 || W != SW || H <= 0 || H % SR || H / SR > 16 || B <= 0 ||
        Cr <= 0 || Cr > 16 || nb <= 0 || nb > FEN_GS_MAXNB)
        return 0;
    if ((size_t)B * H * W * 128 >= (size_t)0x7fff0000) return 0;      // 32-bit buffer offsets
    if (ws_layout(B, H / SR).total >= (size_t)0x7fff0000) return 0;
    return 1;
}

extern "C" size_t fen_group_strip_work_bytes(int B, int H) { return ws_layout(B, H / SR).total; }

extern "C" int fen_group_strip(const fen_group_strip_desc* d, void* stream) {
    if (!d || !d->x || !d->y || !d->work) return FEN_EINVAL;
    if (!fen_group_strip_supported(d->dtype, d->B, d->H, d->W, d->C, d->Cr, d->nb)) return FEN_EUNSUPPORTED;
    if (d->work_bytes < fen_group_strip_work_bytes(d->B, d->H)) return FEN_EINVAL;
    GsArgs a{};
    a.B = d->B, a.H = d->H, a.S = d->H / SR, a.NB = d->nb, a.Cr = d->Cr;
    a.res_scale = d->res_scale, a.inv_hw = 1.0f / (float)(d->H * d->W);
    a.x = d->x, a.y = d->y, a.work = (char*)d->work;
    a.save = d->save ? 1 : 0;
    a.status = d->status, a.fault = d->fault, a.pre_elide = d->pre_elide;
    if (a.save) {
        if (!d->x_last) return FEN_EINVAL;
        a.x_last = d->x_last;
        for (int j = 0; j < d->nb; ++j) {
            if ((j > 0 && !d->sv_x[j]) || !d->sv_z1[j] || !d->sv_a1[j] || !d->sv_t[j] || !d->sv_mean[j] ||
                !d->sv_hid[j] || !d->s_out[j])
                return FEN_EINVAL;
            a.sv_x[j] = d->sv_x[j], a.sv_z1[j] = d->sv_z1[j], a.sv_a1[j] = d->sv_a1[j], a.sv_t[j] = d->sv_t[j];
            a.sv_mean[j] = d->sv_mean[j], a.sv_hid[j] = d->sv_hid[j];
        }
    }
    for (int j = 0; j < d->nb; ++j) {
        if (!d->w1[j] || !d->b1[j] || !d->alpha[j] || !d->w2[j] || !d->b2[j] || !d->fc1[j] || !d->fc2[j])
            return FEN_EINVAL;
        a.w[2 * j] = d->w1[j], a.bias[2 * j] = d->b1[j];
        a.w[2 * j + 1] = d->w2[j], a.bias[2 * j + 1] = d->b2[j];
        a.alpha[j] = d->alpha[j], a.fc1[j] = d->fc1[j], a.fc2[j] = d->fc2[j], a.s_out[j] = d->s_out[j];
    }
    if (!d->wg || !d->bg) return FEN_EINVAL;
    a.w[2 * d->nb] = d->wg, a.bias[2 * d->nb] = d->bg;
    const int grid = d->B * (d->H / SR);
    (void)gs_num_cus();
    hipStream_t s = (hipStream_t)stream;
    if (d->dtype == FEN_F16) {
        if (a.save) launch_gs<f16, true>(a, grid, s);
        else launch_gs<f16, false>(a, grid, s);
    } else {
        if (a.save) launch_gs<bf16, true>(a, grid, s);
        else launch_gs<bf16, false>(a, grid, s);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_group_strip_chain_work_bytes(int B, int H, int ng) {
    if (B <= 0 || H <= 0 || H % SR || ng <= 0) return 0;
    return gs_tab_offset(B, H / SR) + (size_t)(ng + 1) * sizeof(GsTab);     // + the tail's row
}

extern "C" int fen_group_strip_chain_prepare(const fen_group_strip_desc* d, int ng, const fen_group_strip_chain_tail* tail,
                                             void* stream) {
    std::vector<GsTab> tab;
    const int rc = chain_tab(d, ng, tail, tab);
    if (rc != FEN_OK) return rc;
    std::vector<unsigned int> words((sizeof(GsTabHdr) + tab.size() * sizeof(GsTab)) / 4, 0u);
    GsTabHdr hdr{};
    hdr.magic = GS_TAB_MAGIC, hdr.hash = tab_hash(tab), hdr.rows = (int)tab.size();
    memcpy(words.data(), &hdr, sizeof(hdr));
    memcpy((char*)words.data() + sizeof(hdr), tab.data(), tab.size() * sizeof(GsTab));
    unsigned int* dst = (unsigned int*)((char*)d[0].work + gs_tab_offset(d[0].B, d[0].H / SR) - sizeof(GsTabHdr));
    hipStream_t s = (hipStream_t)stream;
    for (size_t o = 0; o < words.size(); o += 896) {
        TabChunk c;
        const int nw = (int)std::min<size_t>(896, words.size() - o);
        memcpy(c.w, words.data() + o, nw * 4);
        hipLaunchKernelGGL(k_tab_write, dim3(1), dim3(256), 0, s, dst + o, c, nw);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_group_strip_chain(const fen_group_strip_desc* d, int ng, const fen_group_strip_chain_tail* tail,
                                     void* stream) {
    std::vector<GsTab> tab;
    const int rc = chain_tab(d, ng, tail, tab);
    if (rc != FEN_OK) return rc;
    const fen_group_strip_desc& d0 = d[0];
    GsArgs a{};
    a.B = d0.B, a.H = d0.H, a.S = d0.H / SR, a.NB = d0.nb, a.Cr = d0.Cr;
    a.res_scale = d0.res_scale, a.inv_hw = 1.0f / (float)(d0.H * d0.W);
    a.work = (char*)d0.work;
    a.status = d0.status, a.fault = d0.fault;
    a.tab = (const GsTab*)((const char*)d0.work + gs_tab_offset(d0.B, d0.H / SR));
    a.tab_hash = tab_hash(tab);
    a.ng = ng;
    a.tail = tail ? 1 : 0;
    a.save = d0.save ? 1 : 0;
    a.pre_elide = d0.pre_elide;
    const int grid = d0.B * (d0.H / SR);
    hipStream_t s = (hipStream_t)stream;
    if (d0.dtype == FEN_F16) {
        if (a.save) launch_gs<f16, true, true>(a, grid, s);
        else launch_gs<f16, false, true>(a, grid, s);
    } else {
        if (a.save) launch_gs<bf16, true, true>(a, grid, s);
        else launch_gs<bf16, false, true>(a, grid, s);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

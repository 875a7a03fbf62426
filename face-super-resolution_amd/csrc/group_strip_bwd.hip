// The backward of one ResidualGroup as ONE persistent launch, its gradients resident on the
// CUs (autograd of reference src/models/blocks.py:185-189: the group conv and its skip, then
// NB x RCAB blocks.py:135-153 with ChannelAttention blocks.py:83-92 in reverse order), the
// counterpart of the forward strip kernel (group_strip.hip) whose saved tensors it reads.
//
// Decomposition as in the forward: one 512-thread block per strip of 8 rows x 64 px, wave w =
// row w, all 64 channels in the MFMA accumulator layout.  Per RCAB j (reverse order), with
// d = dL/d(RCAB j's output) in registers:
//     dt  = d * rs * s_j + g_j                  (the SE backward: g_j from sum(d * t_j))
//     dz1 = conv2^T(dt) * PReLU'(z1_j)          (dalpha partials: sum conv2^T(dt) * z1 * [z1 <= 0])
//     d  <- d + conv1^T(dz1)                    (RCAB j's input gradient, the next d)
// and the group conv's transpose first, d = conv_g^T(dy); at the end dx = d + dy (+ dres).  The
// transposed convs run on the mode-2 (transposed, tap-flipped) packs with the forward's 3-phase
// conv on the LDS image (dt during conv2^T, dz1 during conv1^T; the running conv's 9 taps
// resident, the next conv's streamed in as the phases free their slots).  What crosses CUs, per
// RCAB and strip: the strip's first / last rows of d (the neighbours' dt halo rows are built from
// them) and of dz1 (conv1^T's halo rows), and the strip's partial of sum(d * t) for the next SE
// backward -- the forward's hand-offs (sc1 stores, storing wave's flag, sc1 loads after the poll;
// MI355X_MICROARCH.md inter-workgroup visibility, table row 1), with the same ticketed strips, launch
// epochs, bounded waits (the error word) and counter reset at the end (graph-replayable).
// dt and dz1 go to HBM for the weight gradients (fen_wgrad3x3_multi), the dalpha row partials
// and the SE weight-gradient rows for column sums.
//
// Precision: 16-bit operands, fp32 accumulation; dt, dz1 and every d rounded to the 16-bit
// format where the per-RCAB backward (fen_rcab_bwd + fen_se_bwd_fused) rounds them.  The SE
// backward's sums run over strips (not 16x16 tiles), so results match that path to rounding,
// not bit for bit.
// cache-policy bits of the saved-operand loads and of the dt / dz1 stores (2 = non-temporal):
// default policy both.  Each alone measured faster on one box (5.575-5.627 / 5.596-5.611 vs
// 5.639-5.659 ms), but a 5-way factorial on another (batch m) put saves-nt-only at 5.758-5.770,
// + nt stores 5.783-5.786, + nt loads 5.826-5.845, all three 5.928-5.938 ms: not adopted
#ifndef GSB_LOAD_AUX
#define GSB_LOAD_AUX 0
#endif
#ifndef GSB_SAVE_AUX
#define GSB_SAVE_AUX 0
#endif
#include "strip_common.h"

#include <type_traits>

namespace {

using namespace gs;

constexpr int O_IMG = 0;
constexpr int O_FILT = O_IMG + IMG_BYTES;     // 9 tap slots, slot = kh * 3 + kw
constexpr int O_RED = O_FILT + 9 * TAPB;      // [8 waves][64] f32 row partials of sum(d * t)
constexpr int O_CST = O_RED + 8 * 64 * 4;     // alpha [64] of the running RCAB
constexpr int O_GATE = O_CST + 64 * 4;        // rs * s [64], g [64] of the running RCAB
constexpr int O_SCR = O_GATE + 128 * 4;       // SE backward scratch [64], ticket words
#ifdef FEN_GS_STAMPS
// diagnostic build only (`make gsstamp`, tools/stamp_strip_bwd.py): s_memrealtime stamps of every
// wave in LDS, copied to the workspace's tail at the end; no stamp executes in the product build
constexpr int NSTAMP = 136;
constexpr int O_STAMP = O_SCR + 80 * 4;
constexpr int GSB_LDS = O_STAMP + 8 * NSTAMP * 2;
#define GSTAMP(i)                                                                              \
    do {                                                                                       \
        unsigned long long _rt;                                                                \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_rt)::"memory");        \
        if (lane == 0 && (i) < NSTAMP) stamp_lds[wave * NSTAMP + (i)] = (unsigned short)((unsigned)_rt - t_start); \
    } while (0)
#else
constexpr int GSB_LDS = O_SCR + 80 * 4;
#define GSTAMP(i) \
    do {          \
    } while (0)
#endif
static_assert(GSB_LDS <= 163840, "LDS budget");
// a wave's dt / dz1 save stores (8 per row) are issued last before the wait that follows them
// and left in flight by it (vmcnt(8) instead of vmcnt(0): vector-memory ops retire in issue
// order); GSB_DRAIN_ALL restores the full drains (A/B)
#ifdef GSB_DRAIN_ALL
#define GSB_VMCNT_SAVES(n) asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define GSB_VMCNT_SAVES(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#endif
static_assert(O_FILT % 16 == 0 && O_RED % 16 == 0 && O_GATE % 16 == 0, "alignment");

// workspace: control words, flags, SE partials, boundary rows of d and dz1
struct WsB {
    size_t flg, part, bd, bz, total;
};
__host__ __device__ inline WsB wsb_layout(int B, int S) {
    WsB L;
    size_t o = 256;                          // [0] ticket [1] done [2] error [3] launch epoch
    L.flg = o;  o += (size_t)B * S * 4 * 128;  // per (strip, side, kind) a flag on its own line
    L.part = o; o += (size_t)B * 2 * S * 64 * 8;   // [img][parity][strip][64] {tag, value} granules
    o = (o + 255) & ~(size_t)255;
    const size_t rows = (size_t)B * S * 2 * 2 * ROWB;   // [img][strip][parity][side] rows
    L.bd = o; o += rows;
    L.bz = o; o += rows;
#ifdef FEN_GS_STAMPS
    o += (size_t)B * S * 8 * NSTAMP * 2;            // [block ticket][wave][NSTAMP] u16 (10 ns ticks)
#endif
    L.total = o;
    return L;
}

struct GsbArgs {
    int B, H, S, NB, Cr;
    float res_scale, inv_hw;
    const void* dy;                           // group output gradient [B][H][64][64] NHWC
    void* dx;                                 // group input gradient
    const void* dres;                         // optional extra residual gradient (or NULL)
    const void* w[2 * FEN_GS_MAXNB + 1];      // mode-2 packs in execution order: group conv,
                                              // conv2_{NB-1}, conv1_{NB-1}, ..., conv2_0, conv1_0
    const float* alpha[FEN_GS_MAXNB];
    const float* fc1[FEN_GS_MAXNB];           // [Cr][64]
    const float* fc2[FEN_GS_MAXNB];           // [64][Cr]
    const void* z1[FEN_GS_MAXNB];
    const void* t[FEN_GS_MAXNB];
    const float* s[FEN_GS_MAXNB];
    const float* mean[FEN_GS_MAXNB];
    const float* hid[FEN_GS_MAXNB];
    void* dt[FEN_GS_MAXNB];
    void* dz1[FEN_GS_MAXNB];
    float* dal[FEN_GS_MAXNB];                 // [B*H][64] row partials
    float* dw1p[FEN_GS_MAXNB];                // [B][Cr][64]
    float* dw2p[FEN_GS_MAXNB];                // [B][64][Cr]
    char* work;
    int* status;                              // optional: a timed-out wait is reported here
    int fault;                                // test-only: image 0 strip 1 skips one dz1 flag
    const void* a1[FEN_GS_MAXNB];             // optional: z1 recovered from a1 where every slope > 0
};

template <typename T>
__global__ __launch_bounds__(512, 1) void k_group_strip_bwd(const GsbArgs A) {
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
    int q = lane >> 4, c16 = lane & 15;
    const int B = A.B, H = A.H, NB = A.NB;
    int S = A.S;
    const WsB L = wsb_layout(B, S);
    int* ctl = (int*)A.work;

    if (tid == 0) {
        tick_lds[0] = __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tick_lds[1] = __hip_atomic_load(ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef FEN_GS_STAMPS
        unsigned long long t0;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
        tick_lds[2] = (int)(unsigned)t0;
#endif
    }
    for (int i = tid; i < IMG_BYTES / 16; i += 512) *(uint4*)(img + i * 16) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const int ticket = __builtin_amdgcn_readfirstlane(tick_lds[0]);
    const unsigned epoch = (unsigned)__builtin_amdgcn_readfirstlane(tick_lds[1]);
#ifdef FEN_GS_STAMPS
    const unsigned t_start = (unsigned)__builtin_amdgcn_readfirstlane(tick_lds[2]);   // the block's clock origin
#endif
    GSTAMP(0);
    auto tag_of = [&](int k) -> unsigned { return (epoch << 8) | (unsigned)(k + 1); };
    int im = ticket / S, strip = ticket - im * S;
    int r0 = strip * SR;
    const bool has_up = strip > 0, has_dn = strip + 1 < S;
    const bool bwave = (wave == 0 && has_up) || (wave == SR - 1 && has_dn);
    const int side = wave == 0 ? 0 : 1;
    const int nb_strip = wave == 0 ? strip - 1 : strip + 1;
    // dt's halo rows are built by four waves per side (a quarter row each: 2 of the 8 chunks
    // per lane): waves 0-3 the upper row, waves 4-7 the lower one
    constexpr int HK = 2;
    const int hs = wave < 4 ? 0 : 1;
    const bool hwave = hs == 0 ? has_up : has_dn;
    const int hk0 = HK * (wave & 3);

    const size_t act_bytes = (size_t)B * H * SW * 128;
    const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc((void*)A.work, 0, (int)L.total, 0x00020000);
    unsigned* flg = (unsigned*)(A.work + L.flg);
    // one flag word per (strip, side, kind), own 128-B line: kind 0 = dz1 row, 1 = d row
    auto flag_of = [&](int s_, int sd, int kind) -> unsigned* { return flg + (((im * S + s_) * 2 + sd) * 2 + kind) * 32; };
    auto rowoff = [&](size_t base, int s_, int par, int sd) -> int {
        return (int)(base + ((size_t)((im * S + s_) * 2 + par) * 2 + sd) * ROWB);
    };

    auto issue_taps = [&](int ci, int k0, int n) {     // taps k0 .. k0 + n - 1 of conv ci -> slots
        const i32x4 wr = make_rsrc(A.w[ci], 9u * 64u * 128u);
        int ll = lane;
        asm volatile("" : "+v"(ll));
        const int s = wave * 64 + ll, r = s >> 3, pc = s & 7;
        const int v0 = (r * 64 + ((pc ^ ((r >> 1) & 7)) * 8)) * 2;
        for (int k = k0; k < k0 + n; ++k)
            dma16(wr, __builtin_amdgcn_readfirstlane(lds_addr(filt + k * TAPB + wave * 1024)), v0 + k * TAPB);
    };
    auto issue_kh1 = [&](int ci) { issue_taps(ci, 3, 3); };
    auto issue_kh02 = [&](int ci) {
        issue_taps(ci, 0, 3);
        issue_taps(ci, 6, 3);
    };

    // accumulator layout: lane (q, c16) holds channels 16m + 4q + i of pixel 16p + c16
    auto px_off = [&](int row, int p) -> size_t { return ((size_t)(im * H + row) * SW + 16 * p + c16) * 128; };
    // the wave's row of a [B,H,64,64] tensor into the accumulator layout: one lane offset
    // (from opaque lane coordinates), (m, p) as immediate offsets
    auto load_acc = [&](const void* base, uint2 (&v)[4][4]) {
        const void* bp = base;
        asm volatile("" : "+s"(bp));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)bp, 0, (int)act_bytes, 0x00020000);
        int qq = q, cc = c16;
        asm volatile("" : "+v"(qq), "+v"(cc));
        const int lb = (int)((size_t)(im * H + r0 + wave) * SW * 128) + cc * 128 + qq * 8;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p)
                v[m][p] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, lb + p * 2048 + m * 32, 0, GSB_LOAD_AUX));
    };
    auto write_row_lds = [&](int lrow, const uint2 (&v)[4][4]) {
        int qq = q, cc = c16;
        asm volatile("" : "+v"(qq), "+v"(cc));
        const int key = (cc + 1) & 7;
        char* rb = img + lrow * IROW + (cc + 1) * 128 + (qq & 1) * 8;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            char* mb = rb + (((2 * m + (qq >> 1)) ^ key) << 4);
#pragma unroll
            for (int p = 0; p < 4; ++p) *(uint2*)(mb + p * 2048) = v[m][p];
        }
    };
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
    // dt / dz1 for the group's weight gradients (the next launch); GSB_SAVE_AUX: their stores'
    // cache-policy bits (A/B: 2 = non-temporal)
    auto save_row = [&](void* base, const uint2 (&v)[4][4]) {
        void* bp = base;
        asm volatile("" : "+s"(bp));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(bp, 0, (int)act_bytes, 0x00020000);
        store_row(rs, (int)((size_t)(im * H + r0 + wave) * SW * 128), v, GSB_SAVE_AUX);
    };
    auto halo_to_lds = [&](int lrow, const uint4 (&v)[8]) {
        int ll = lane;
        asm volatile("" : "+v"(ll));
        char* hb = img + lrow * IROW + hcol((ll >> 3) + 1, ll & 7);
#pragma unroll
        for (int k = 0; k < 8; ++k) *(uint4*)(hb + k * 1024) = v[k];
    };
    auto load_row = [&](int off, uint4 (&v)[8]) {           // sc1: a handed-off row
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wsr, off + (lane + 64 * k) * 16, 0, 16));
    };

    // ================= start-up: the group conv's taps, dy's strip (+ halo rows) in LDS =========
    issue_taps(0, 0, 9);
    {
        uint2 v[4][4];
        load_acc(A.dy, v);
        if (bwave) {
            const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc((void*)A.dy, 0, (int)act_bytes, 0x00020000);
            uint4 hv[8];
            const int row = wave == 0 ? r0 - 1 : r0 + SR;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                hv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      yrs, (int)(((size_t)(im * H + row) * SW) * 128) + (lane + 64 * k) * 16, 0, 0));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            halo_to_lds(wave == 0 ? 0 : SR + 1, hv);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        write_row_lds(wave + 1, v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();                                        // the group conv's taps landed; dy's image complete

    // ================= step k: k = 0 the group conv^T; k >= 1 RCAB jr = NB - k =================
    // Per RCAB: B_X (dt image complete), B_E (conv2^T done), B_Y (dz1 image complete), B_Z (the
    // strip's sum(d * t) rows complete, conv1^T done), B_G (the next RCAB's SE backward known).
    uint2 dr[4][4];                                         // d, packed 16-bit
    const int khP2 = wave == 0 ? 2 : 0, khP3 = 2 - khP2;   // wave 0's upper halo row is read last
    bool ok = true;
    float cv = 0.f;
    for (int k = 0; k <= NB; ++k) {
        const int jr = NB - k;                              // k >= 1: this step's RCAB
        const int par = k & 1;
        const int sb = 2 + 12 * k;                          // this step's stamp slots
        GSTAMP(sb);
        {
            int ll = lane;
            asm volatile("" : "+v"(ll), "+s"(im), "+s"(strip), "+s"(S), "+s"(r0));
            lane = ll, q = ll >> 4, c16 = ll & 15;
        }
        f32x4 acc[4][4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[m][p] = zero4();
        uint2 tv[4][4];                                     // t_{jr-1} (or dy at the end) for the step's epilogue
        if (k == 0) {
            // ---- the group conv^T on dy (its image and halo rows complete since start-up)
            conv_phase<T>(acc, img, filt, 1, wave, q, c16);
            __syncthreads();                                // B_X: kh = 1 slots free
            issue_kh1(1);                                   // conv2^T of RCAB NB-1
            load_acc(A.t[NB - 1], tv);
            conv_phase<T>(acc, img, filt, khP2, wave, q, c16);
            conv_phase<T>(acc, img, filt, khP3, wave, q, c16);
        } else {
            const int ci = 2 * k - 1;
#ifdef GSB_OLD_START
            issue_kh02(ci);                                 // conv2^T's kh = 0, 2 taps (slots free since B_G)
#endif
            if (wave == 2) cst[lane] = cv;                  // alpha of RCAB jr, read after B_E
            uint4 nd[HK];
            if (hwave) {
                // the neighbour's d row (this wave's part): lands during phase 1.  No flag poll: its
                // storing wave drained the row before its B_Z, after which its block published the SE
                // partial that wave 1's sweep saw before this block's B_G (the hand-off's signal)
                const int ns = hs == 0 ? strip - 1 : strip + 1;
                const int od = rowoff(L.bd, ns, (k - 1) & 1, 1 - hs) + (lane + 64 * hk0) * 16;
#pragma unroll
                for (int kk = 0; kk < HK; ++kk)
                    nd[kk] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wsr, od + kk * 1024, 0, 16));
            }
#ifndef GSB_OLD_START
            // after the poll (a poll waits on every older vector-memory op of its wave; the
            // neighbour's flag was set before its B_Z, so before this block passed B_G)
            issue_kh02(ci);                                 // conv2^T's kh = 0, 2 taps (slots free since B_G)
#endif
            // ---- dt = d * rs * s + g (as stored, 16-bit): the LDS image's own row, HBM for the
            // weight gradient
            uint2 dv[4][4];
            {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float4 ga = *(const float4*)(gate + 16 * m + 4 * q);
                    const float4 gb = *(const float4*)(gate + 64 + 16 * m + 4 * q);
#pragma unroll
                    for (int p = 0; p < 4; ++p)
                        dv[m][p] = pk4<T>(lo16<T>(dr[m][p].x) * ga.x + gb.x, hi16<T>(dr[m][p].x) * ga.y + gb.y,
                                          lo16<T>(dr[m][p].y) * ga.z + gb.z, hi16<T>(dr[m][p].y) * ga.w + gb.w);
                }
                write_row_lds(wave + 1, dv);
            }
            // dt's row out for the weight gradient: issued after every op the wait below needs,
            // and left in flight by it (vector-memory ops retire in issue order)
            asm volatile("" ::: "memory");
            save_row(A.dt[jr], dv);
            // ================= conv2^T =================
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            GSTAMP(sb + 1);
            conv_phase<T>(acc, img, filt, 1, wave, q, c16);
            GSTAMP(sb + 2);
            GSB_VMCNT_SAVES(8);                                 // this conv's taps; the halo rows (dt's save in flight)
            if (hwave) {                                    // its half of dt's halo row, same arithmetic
                const float4 ga = *(const float4*)(gate + (lane & 7) * 8);
                const float4 gb = *(const float4*)(gate + (lane & 7) * 8 + 4);
                const float4 ha = *(const float4*)(gate + 64 + (lane & 7) * 8);
                const float4 hb4 = *(const float4*)(gate + 64 + (lane & 7) * 8 + 4);
                const float g8[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
                const float h8[8] = {ha.x, ha.y, ha.z, ha.w, hb4.x, hb4.y, hb4.z, hb4.w};
                char* hb = img + (hs == 0 ? 0 : SR + 1) * IROW + hcol((lane >> 3) + 1, lane & 7) + hk0 * 1024;
#pragma unroll
                for (int kk = 0; kk < HK; ++kk) {
                    float df[8], yv[8];
                    unpack16<T>(nd[kk], df);
#pragma unroll
                    for (int e = 0; e < 8; ++e) yv[e] = df[e] * g8[e] + h8[e];
                    *(uint4*)(hb + kk * 1024) = pack16<T>(yv);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            __syncthreads();                                // B_X: dt's image complete; kh = 1 slots free
            GSTAMP(sb + 3);
            issue_kh1(ci + 1);                              // conv1^T's kh = 1 taps
            uint2 zv[4][4];
            // PReLU's input, for the epilogue: z1, or a1 when every slope of RCAB jr is > 0 (the
            // forward's pre_elide may not have written z1 then; lane = channel)
            const bool recz = A.a1[jr] != nullptr && __ballot(cst[lane] > 0.f) == ~0ull;
            load_acc(recz ? A.a1[jr] : A.z1[jr], zv);
            conv_phase<T>(acc, img, filt, khP2, wave, q, c16);
            conv_phase<T>(acc, img, filt, khP3, wave, q, c16);
            GSTAMP(sb + 4);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // ---- dz1 = conv2^T(dt) * PReLU'(z1) -> LDS (own row), boundary row out, HBM; the
            // row's dalpha partials sum conv2^T(dt) * z1 * [z1 <= 0] (blocks.py:146's PReLU).
            // Computed before B_E (only the LDS write must wait for every wave's dt reads): a wave
            // done with its phases works while its SIMD partner still issues MFMAs
#ifdef GSB_LATE_EPI
            __syncthreads();                                // A/B variant: the epilogue after every wave's conv
#endif
            uint2 zd[4][4];
            float* dal = A.dal[jr];
            asm volatile("" : "+s"(dal));
            {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float4 aa = *(const float4*)(cst + 16 * m + 4 * q);
                    const float alp[4] = {aa.x, aa.y, aa.z, aa.w};
                    float ds[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        // recz: a1 has z1's sign (PReLU' is exact); the slope partial sums
                        // g * a1 over a1 <= 0, i.e. alpha times the z1 sum: scaled by 1 / alpha below
                        const float z[4] = {lo16<T>(zv[m][p].x), hi16<T>(zv[m][p].x), lo16<T>(zv[m][p].y),
                                            hi16<T>(zv[m][p].y)};
                        float v[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            v[i] = prelu_bwd_f(acc[m][p][i], z[i], alp[i]);
                            ds[i] += prelu_dalpha_f(acc[m][p][i], z[i]);
                        }
                        zd[m][p] = pk4<T>(v[0], v[1], v[2], v[3]);
                    }
                    float sv[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) sv[i] = group16_sum(ds[i]) * (recz ? __builtin_amdgcn_rcpf(alp[i]) : 1.f);
                    // the row's partial -> red[wave] (free since the previous step's publish); the
                    // strip's sum over its 8 rows goes out after B_E (8x fewer rows to column-sum)
                    if (c16 == 0) *(float4*)(red + wave * 64 + 16 * m + 4 * q) = make_float4(sv[0], sv[1], sv[2], sv[3]);
                }
            }
            GSTAMP(sb + 5);
            __syncthreads();                                // B_E: dt's reads done (all slots free); taps visible
            GSTAMP(sb + 6);
            issue_kh02(ci + 1);
            if (wave == 2) {                                // the strip's dalpha partial, rows in order (before B_Y)
                float a = 0.f;
#pragma unroll
                for (int w = 0; w < SR; ++w) a += red[w * 64 + lane];
                dal[(size_t)(im * S + strip) * 64 + lane] = a;
            }
            write_row_lds(wave + 1, zd);
            if (bwave) store_row(wsr, rowoff(L.bz, strip, par, side), zd, 16);
            asm volatile("" ::: "memory");
            save_row(A.dz1[jr], zd);
            // ================= conv1^T =================
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int p = 0; p < 4; ++p) acc[m][p] = zero4();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            GSTAMP(sb + 7);
            conv_phase<T>(acc, img, filt, 1, wave, q, c16);     // own dz1 row only: no barrier
            GSTAMP(sb + 8);
            GSB_VMCNT_SAVES(8);                                 // conv1^T's other taps; the dz1 boundary stores
            if (bwave && lane == 0 && !(A.fault && ticket == 1 && k == 1 && side == 0))
                __hip_atomic_store(flag_of(strip, side, 0), tag_of(k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();                                // B_Y: dz1's image complete; kh = 1 slots free
#ifdef GSB_NEW_HALO
            // the boundary waves poll for the neighbour's dz1 row first (its flag follows its own
            // phase 1, like this block's B_Y) and load it before the tap DMA and t: the poll then
            // waits on no other load, and the row lands during phase 2
            uint4 hv[8];
            if (bwave) {
                ok = ok && poll_eq(flag_of(nb_strip, 1 - side, 0), tag_of(k));
                load_row(rowoff(L.bz, nb_strip, par, 1 - side), hv);
            }
            if (jr > 0) issue_kh1(ci + 2);                  // the next RCAB's conv2^T
            load_acc(jr > 0 ? A.t[jr - 1] : A.dy, tv);
            conv_phase<T>(acc, img, filt, khP2, wave, q, c16);
            if (bwave) {                                    // -> this wave's private halo row
                halo_to_lds(wave == 0 ? 0 : SR + 1, hv);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
#else
            if (jr > 0) issue_kh1(ci + 2);                  // the next RCAB's conv2^T
            load_acc(jr > 0 ? A.t[jr - 1] : A.dy, tv);
            conv_phase<T>(acc, img, filt, khP2, wave, q, c16);
            if (bwave) {
                // the neighbour's dz1 row -> this wave's private halo row
                ok = ok && poll_eq(flag_of(nb_strip, 1 - side, 0), tag_of(k));
                uint4 hv[8];
                load_row(rowoff(L.bz, nb_strip, par, 1 - side), hv);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                halo_to_lds(wave == 0 ? 0 : SR + 1, hv);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
#endif
            conv_phase<T>(acc, img, filt, khP3, wave, q, c16);
            GSTAMP(sb + 9);
        }
        if (k > 0 && jr == 0) {
            // ---- the group input's gradient: d + conv1^T(dz1) + dy (the group's skip) (+ dres)
            // (fp32 sums in acc, one rounding; dres loaded into tv's registers once dy is in)
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    acc[m][p][0] += lo16<T>(dr[m][p].x) + lo16<T>(tv[m][p].x);
                    acc[m][p][1] += hi16<T>(dr[m][p].x) + hi16<T>(tv[m][p].x);
                    acc[m][p][2] += lo16<T>(dr[m][p].y) + lo16<T>(tv[m][p].y);
                    acc[m][p][3] += hi16<T>(dr[m][p].y) + hi16<T>(tv[m][p].y);
                }
            if (A.dres) {
                load_acc(A.dres, tv);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        acc[m][p][0] += lo16<T>(tv[m][p].x), acc[m][p][1] += hi16<T>(tv[m][p].x);
                        acc[m][p][2] += lo16<T>(tv[m][p].y), acc[m][p][3] += hi16<T>(tv[m][p].y);
                    }
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int p = 0; p < 4; ++p) dr[m][p] = pk4<T>(acc[m][p][0], acc[m][p][1], acc[m][p][2], acc[m][p][3]);
            save_row(A.dx, dr);
            break;
        }
        // ---- the next d: conv^T(..) (+ d), boundary row out; its row sums of d * t_{jn} (the SE
        // backward's operand of RCAB jn = NB - 1 - k) -> red[wave]
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                float v[4] = {acc[m][p][0], acc[m][p][1], acc[m][p][2], acc[m][p][3]};
                if (k > 0) {
                    v[0] += lo16<T>(dr[m][p].x), v[1] += hi16<T>(dr[m][p].x);
                    v[2] += lo16<T>(dr[m][p].y), v[3] += hi16<T>(dr[m][p].y);
                }
                dr[m][p] = pk4<T>(v[0], v[1], v[2], v[3]);
            }
        if (bwave) store_row(wsr, rowoff(L.bd, strip, par, side), dr, 16);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float ds[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                ds[0] += lo16<T>(dr[m][p].x) * lo16<T>(tv[m][p].x);
                ds[1] += hi16<T>(dr[m][p].x) * hi16<T>(tv[m][p].x);
                ds[2] += lo16<T>(dr[m][p].y) * lo16<T>(tv[m][p].y);
                ds[3] += hi16<T>(dr[m][p].y) * hi16<T>(tv[m][p].y);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float s = group16_sum(ds[i]);
                if (c16 == 0) red[wave * 64 + 16 * m + 4 * q + i] = s;
            }
        }
        const int jn = NB - 1 - k;                          // the next step's RCAB
        if (wave == 2) cv = A.alpha[jn][lane];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the d row drained before B_Z (see the step start)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GSTAMP(sb + 10);
        __syncthreads();                                    // B_Z: the row sums in red; conv reads done (all slots free)
        if (wave == 3) {
            // the strip's partial as {tag, value} granules (one 8-B sc1 store each), rows in order
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < SR; ++w) s += red[w * 64 + lane];
            unsigned long long* pg = (unsigned long long*)(A.work + L.part) + ((size_t)(im * 2 + par) * S + strip) * 64 + lane;
            __hip_atomic_store(pg, ((unsigned long long)tag_of(k) << 32) | __float_as_uint(s), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (wave == 1) {
            // SE backward of RCAB jn (autograd of blocks.py:88-92 and the scaled residual
            // blocks.py:153): a = sum over the image of d * t (the strips' granules in strip
            // order), dz = a * rs * s (1 - s) through the sigmoid, dh = [hid > 0] FC2^T dz,
            // FC weight-gradient rows dz x hid and dh x mean (this image's, written by strip 0),
            // g = FC1^T dh / HW; then the gate area holds rs * s and g for dt = d * rs * s + g
            int ll = lane;
            asm volatile("" : "+v"(ll));                    // lane-derived values computed here, not hoisted
            const int Cr = A.Cr, jj = ll & 15, qq = ll >> 4;
            const float* f1p = A.fc1[jn];
            const float* f2p = A.fc2[jn];
            const float* sp = A.s[jn];
            const float* mp = A.mean[jn];
            const float* hp = A.hid[jn];
            asm volatile("" : "+s"(f1p), "+s"(f2p), "+s"(sp), "+s"(mp), "+s"(hp));
            const __amdgpu_buffer_rsrc_t f1r = __builtin_amdgcn_make_buffer_rsrc((void*)f1p, 0, Cr * 64 * 4, 0x00020000);
            const __amdgpu_buffer_rsrc_t f2r = __builtin_amdgcn_make_buffer_rsrc((void*)f2p, 0, Cr * 64 * 4, 0x00020000);
            float w1c[16], w2r[16];                         // fc1[jj'][lane] (jj' < 16), fc2[16 qq + kk][jj]
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                w1c[kk] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(f1r, (kk * 64 + ll) * 4, 0, 0));
                w2r[kk] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(f2r, ((16 * qq + kk) * Cr + jj) * 4, 0, 0));
            }
            const float sv = sp[im * 64 + ll];
            const float mv = mp[im * 64 + ll];
            const float hv = jj < Cr ? hp[im * Cr + jj] : 0.f;
            const unsigned tg = tag_of(k);
            const int po = (int)(L.part + ((size_t)(im * 2 + par) * S) * 512) + ll * 8;   // this image's granules
            float asum = 0.f;
            bool got = false;
            // the strips' granules swept 8 at a time (one round of 8 loads when S <= 8, two in
            // order when S <= 16): 8 live granules on this wave's path instead of 16 (GSB_POLL16:
            // all 16 loads in flight at once, strips past S re-reading strip 0)
#ifndef GSB_POLL16
            constexpr int NSW = 8;
#else
            constexpr int NSW = 16;
#endif
            for (int it = 0; it < SPIN_MAX && ok; ++it) {
                unsigned bad = 0u;
                float ms = 0.f;                             // in strip order
                for (int s0 = 0; s0 < S; s0 += NSW) {
                    asm volatile("" ::: "memory");          // a fresh sc1 load per poll
                    uint2 gv[NSW];
#pragma unroll
                    for (int s_ = 0; s_ < NSW; ++s_)
                        gv[s_] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                               wsr, po + (s0 + s_ < S ? s0 + s_ : 0) * 512, 0, 16));
#pragma unroll
                    for (int s_ = 0; s_ < NSW; ++s_) {
                        const bool in = s0 + s_ < S;
                        ms += in ? __uint_as_float(gv[s_].x) : 0.f;
                        bad |= (unsigned)(in & (gv[s_].y != tg));
                    }
                }
                asum = ms;
                if (__all(bad == 0u)) {
                    got = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            ok = ok && got;
            const float rs = A.res_scale;
            const float dz = asum * rs * sv * (1.f - sv);
            scr[ll] = dz;
            float h = 0.f;
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) h += w2r[kk] * scr[16 * qq + kk];
            h += __shfl_xor(h, 16, 64);
            h += __shfl_xor(h, 32, 64);
            const float dh = (jj < Cr && hv > 0.f) ? h : 0.f;    // lanes jj (every qq) hold dh[jj]
            float g = 0.f;
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) g += w1c[kk] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dh), kk));
            gate[ll] = rs * sv;
            gate[64 + ll] = g * A.inv_hw;
            if (strip == 0) {
                // this image's rows (buffer stores: offsets past Cr rows fall outside the range)
                float* d1p = A.dw1p[jn];
                float* d2p = A.dw2p[jn];
                asm volatile("" : "+s"(d1p), "+s"(d2p));
                const __amdgpu_buffer_rsrc_t d1r =
                    __builtin_amdgcn_make_buffer_rsrc(d1p + (size_t)im * Cr * 64, 0, Cr * 64 * 4, 0x00020000);
                const __amdgpu_buffer_rsrc_t d2r =
                    __builtin_amdgcn_make_buffer_rsrc(d2p + (size_t)im * 64 * Cr, 0, Cr * 64 * 4, 0x00020000);
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {
                    const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dh), kk)) * mv;
                    const float a2 = dz * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hv), kk));
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a1), d1r, (kk * 64 + ll) * 4, 0, 0);
                    // [64][Cr]: column kk of row lane, dropped for kk >= Cr
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a2), d2r, kk < Cr ? (ll * Cr + kk) * 4 : Cr * 256,
                                                          0, 0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GSTAMP(sb + 11);
        __syncthreads();                                    // B_G: the next RCAB's rs * s and g in LDS
    }
    GSTAMP(NSTAMP - 1);
    // ---- the last block out advances the epoch and resets the ticket counters for the next launch
    if (!ok) __hip_atomic_fetch_or(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) strip_finish(ctl, B * S, A.status, FEN_STATUS_GS_BWD);
#ifdef FEN_GS_STAMPS
    __syncthreads();
    {
        unsigned short* dst = (unsigned short*)(A.work + L.bz + (size_t)B * S * 2 * 2 * ROWB) + (size_t)ticket * 8 * NSTAMP;
        for (int i = tid; i < 8 * NSTAMP; i += 512) dst[i] = stamp_lds[i];
    }
#endif
}

template <typename T>
void launch_gsb(const GsbArgs& a, int grid, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_group_strip_bwd<T>, hipFuncAttributeMaxDynamicSharedMemorySize, GSB_LDS);
        attr = true;
    }
    hipLaunchKernelGGL(k_group_strip_bwd<T>, dim3(grid), dim3(512), GSB_LDS, s, a);
}

}  // namespace

extern "C" size_t fen_group_strip_bwd_work_bytes(int B, int H) { return wsb_layout(B, H / SR).total; }

extern "C" int fen_group_strip_bwd_dal_rows(int B, int H) { return B * (H / SR); }

extern "C" int fen_group_strip_bwd_supported(int dtype, int B, int H, int W, int C, int Cr, int nb) {
    if (!fen_group_strip_supported(dtype, B, H, W, C, Cr, nb)) return 0;
    if (wsb_layout(B, H / SR).total >= (size_t)0x7fff0000) return 0;
    return 1;
}

extern "C" int fen_group_strip_bwd(const fen_group_strip_bwd_desc* d, void* stream) {
    if (!d || !d->dy || !d->dx || !d->work || !d->wgt) return FEN_EINVAL;
    if (!fen_group_strip_bwd_supported(d->dtype, d->B, d->H, d->W, d->C, d->Cr, d->nb)) return FEN_EUNSUPPORTED;
    if (d->work_bytes < fen_group_strip_bwd_work_bytes(d->B, d->H)) return FEN_EINVAL;
    if (d->dx == d->dy || (d->dres && d->dres == d->dx)) return FEN_EINVAL;
    GsbArgs a{};
    const int nb = d->nb;
    a.B = d->B, a.H = d->H, a.S = d->H / SR, a.NB = nb, a.Cr = d->Cr;
    a.res_scale = d->res_scale, a.inv_hw = 1.0f / (float)(d->H * d->W);
    a.dy = d->dy, a.dx = d->dx, a.dres = d->dres, a.work = (char*)d->work;
    a.status = d->status, a.fault = d->fault;
    a.w[0] = d->wgt;
    for (int j = 0; j < nb; ++j) {
        if (!d->w1t[j] || !d->w2t[j] || !d->alpha[j] || !d->fc1[j] || !d->fc2[j] || !d->z1[j] || !d->t[j] ||
            !d->s[j] || !d->mean[j] || !d->hid[j] || !d->dt[j] || !d->dz1[j] || !d->dalpha_part[j] || !d->dw1p[j] ||
            !d->dw2p[j])
            return FEN_EINVAL;
        const int k = nb - j;                     // RCAB j runs in step k
        a.w[2 * k - 1] = d->w2t[j], a.w[2 * k] = d->w1t[j];
        a.alpha[j] = d->alpha[j], a.fc1[j] = d->fc1[j], a.fc2[j] = d->fc2[j];
        a.z1[j] = d->z1[j], a.t[j] = d->t[j], a.s[j] = d->s[j], a.mean[j] = d->mean[j], a.hid[j] = d->hid[j];
        a.a1[j] = d->a1[j];
        a.dt[j] = d->dt[j], a.dz1[j] = d->dz1[j], a.dal[j] = d->dalpha_part[j];
        a.dw1p[j] = d->dw1p[j], a.dw2p[j] = d->dw2p[j];
    }
    const int grid = d->B * (d->H / SR);
    hipStream_t s = (hipStream_t)stream;
    if (d->dtype == FEN_F16) launch_gsb<f16>(a, grid, s);
    else launch_gsb<bf16>(a, grid, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// 128-channel RCAB convs (BASELINE configs[4]: FaceEnhanceNet with num_channels = 128, Cr = 32,
// reference src/models/blocks.py:105-153 (RCAB), blocks.py:83-92 (ChannelAttention),
// blocks.py:185-189 (ResidualGroup)), one persistent launch per conv with the RCAB's elementwise
// work folded into its prologue / epilogue:
//   mode 1 (conv1):      in  = x_j = x_{j-1} + rs * s_{j-1} * t_{j-1}   (deferred gate; or x_j)
//                        out = a1 = PReLU(conv1(x_j) + b1)   (+ x_j's own tile, for the next RCAB)
//   mode 2 (conv2):      in  = a1;  out = t_j = conv2(a1) + b2  + per-tile channel sums of t_j
//   mode 3 (group conv): in  = the chain's output (deferred gate as mode 1); out = conv + b + res
//   mode 4 (upsampler stage, custom.py's conv(C -> 4C) + PixelShuffle(2) + PReLU): the 4C
//                        outputs as 4 blocks of 128 (the shuffle-permuted mode-1 pack: block k =
//                        sub-pixel (k >> 1, k & 1)), run one after another on the tile's image
// The gate s_{j-1} of an image (mean over its tiles' sums -> FC1 -> ReLU -> FC2 -> sigmoid) is
// recomputed by every block in its prologue from the producer's tile sums: the kernel boundary is
// the per-image hand-off, no block ever waits on another (any grid, graph-replayable).
//
// Tile = 4 rows x 64 px x 128 output channels; one 512-thread block per CU walks tiles
// (grid = min(tiles, CUs); the stress config's 128x128 B=4 is exactly one tile per CU), wave w =
// (row w >> 1, output-channel half w & 1): 64 px x 64 co, 16 accumulator tiles of
// v_mfma_f32_16x16x32_{f16,bf16}, the group-strip kernel's per-wave shape.  LDS:
//   * the input image: 6 rows (tile + halo) x 66 columns x 256 B (128 ch), 99 KB; 16-B chunk c
//     of column col at chunk c ^ (col & 15) (16 consecutive columns at one chunk -> 16 distinct
//     slots of the 256-B bank row);
//   * a 3-slot filter ring: a slot = one (tap, 64-input-channel half) = [128 co][64 ci], 16 KB,
//     filled by LDS-DMA two steps ahead (18 steps per conv, one barrier each).  128x128x9 filters
//     (295 KB) do not fit beside the image.
// Precision: 16-bit operands, fp32 accumulation; x_j, a1, t rounded to the 16-bit format where
// the per-op path (conv + fen_se_fused) rounds them.
#include "fen_common.h"

namespace {

constexpr int TR = 4, TW = 64, CC = 128;
constexpr int ICOL = TW + 2;                 // 66 image columns
constexpr int PXB = CC * 2;                  // 256 B per pixel
constexpr int IROW = ICOL * PXB;             // 16896 B per image row
constexpr int IMG = (TR + 2) * IROW;         // 101376 B = 99 DMA pieces
constexpr int NUNIT = IMG / 16;              // 6336 16-B units
constexpr int NPIECE = IMG / 1024;           // 99
constexpr int SLOT = CC * 128;               // [128 co][64 ci] 16-bit
constexpr int NSLOT = 3;
constexpr int NSTEP = 18;                    // 9 taps x 2 input-channel halves
constexpr int O_RING = IMG;
constexpr int O_CST = O_RING + NSLOT * SLOT; // bias [4][128] (mode 4: per output block), alpha [128]
constexpr int O_GATE = O_CST + 5 * CC * 4;   // rs * s [128]
constexpr int O_RED = O_GATE + CC * 4;       // [4][128] f32
constexpr int O_SCR = O_RED + 4 * CC * 4;    // mean [128], hid [32]
constexpr int LDS128 = O_SCR + (CC + 32) * 4;
static_assert(LDS128 <= 163840, "LDS budget");
static_assert(IMG % 1024 == 0, "whole DMA pieces");
constexpr unsigned OOB = 0x80000000u;        // a buffer offset past every tensor: loads return 0

struct K128 {
    int B, H, W, Cr;
    float res_scale, inv_hw;
    const void* x;        // conv input (mode 2: a1), or x_{j-1} with tp
    const void* tp;       // t_{j-1} (deferred gate) or NULL
    const float* pp;      // tile sums of t_{j-1} [B][tiles][128]
    const float* pfc1;    // [Cr][128]
    const float* pfc2;    // [128][Cr]
    float* ps;            // s_{j-1} [B][128] copy or NULL
    void* xo;             // x_j out or NULL
    const void* w;        // packed mode 0 [9][128][128]
    const float* bias;
    const float* alpha;
    const void* res;      // mode 3
    void* y;
    void* z1;             // mode 1, optional
    float* part;          // mode 2
};

// s_waitcnt vmcnt(n) for the few counts the step loop needs
__device__ __forceinline__ void vm_wait(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

template <typename T>
__device__ __forceinline__ uint2 pk4(float a, float b, float c, float d) {
    return make_uint2(pack2<T>(a, b), pack2<T>(c, d));
}
// lanes q and q ^ 1 trade a 4-channel half so each holds 8 consecutive channels (chunk_of)
__device__ __forceinline__ uint4 pair16(uint2 lo, uint2 hi) {
    const auto a = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
    return make_uint4(a[0], b[0], a[1], b[1]);
}
__device__ __forceinline__ int chunk_of(int mp, int q) { return 4 * mp + ((q & 1) ? 2 : 0) + (q >> 1); }

template <typename T, int MODE, bool COMB>
__global__ __launch_bounds__(512, 1) void k_rcab128(const K128 A) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* img = smem;
    char* ring = smem + O_RING;
    float* cst = (float*)(smem + O_CST);
    float* gate = (float*)(smem + O_GATE);
    float* red = (float*)(smem + O_RED);
    float* scr = (float*)(smem + O_SCR);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = wave_id();
    const int wr = wave >> 1, wh = wave & 1;          // the wave's output row and channel half
    const int B = A.B, H = A.H, W = A.W;
    const int tpr = W / TW, tpi = (H / TR) * tpr, ntiles = B * tpi;
    const unsigned act_bytes = (unsigned)((size_t)B * H * W * PXB);
    constexpr int NCO = MODE == 4 ? 4 : 1;           // 128-channel output blocks per tile
    constexpr int NG = NCO * NSTEP;                   // filter steps per tile
    const i32x4 wrs = make_rsrc(A.w, 9u * NCO * CC * CC * 2u);

    // filter step g = (output block g / 18; tap (g % 18) >> 1, input half g & 1) into ring slot
    // g % 3: this wave's 2 pieces (packed [9][NCO * 128][128])
    // the step loop's addresses from per-lane parts computed once per tile, after the staging
    // (their registers are not live through it): the two DMA pieces' source offsets, the A
    // (filter slot) and B (image, per kw) fragment offsets of k-half 0.  The chunk index
    // 8 ch + 4 ks + q has ch, ks in bits the lane's q does not touch, and the row / column parts
    // are multiples of 128 / 256 B, so the (ch, ks) forms are those XORed with (4 ks + 8 ch) << 4
    int dlane0 = 0, dlane1 = 0, aoff0 = 0, boffA = 0, boffB = 0, boffC = 0;
    auto lane_offsets = [&]() {
        int ll = lane;
        asm volatile("" : "+v"(ll));
        const int u0 = (2 * wave) * 64 + ll, r0_ = u0 >> 3, r1_ = r0_ + 8, pc = u0 & 7;
        dlane0 = (r0_ * CC + (pc ^ ((r0_ >> 1) & 7)) * 8) * 2;
        dlane1 = (r1_ * CC + (pc ^ ((r1_ >> 1) & 7)) * 8) * 2;
        const int q = ll >> 4, c16 = ll & 15;
        aoff0 = (64 * wh + c16) * 128 + ((q ^ ((c16 >> 1) & 7)) << 4);
        boffA = wr * IROW + c16 * PXB + ((q ^ (c16 & 15)) << 4);
        boffB = wr * IROW + (c16 + 1) * PXB + ((q ^ ((c16 + 1) & 15)) << 4);
        boffC = wr * IROW + (c16 + 2) * PXB + ((q ^ ((c16 + 2) & 15)) << 4);
    };
    auto issue_step_fast = [&](int g) {
        const int cb = g / NSTEP, s = g - cb * NSTEP;
        const int tap = s >> 1, ch = s & 1;
        char* slot = ring + (g % NSLOT) * SLOT;
        const int sbase = ((tap * NCO + cb) * CC * CC + ch * 64) * 2;
        dma16(wrs, __builtin_amdgcn_readfirstlane(lds_addr(slot + (2 * wave) * 1024)), sbase + dlane0);
        dma16(wrs, __builtin_amdgcn_readfirstlane(lds_addr(slot + (2 * wave + 1) * 1024)), sbase + dlane1);
    };
    auto issue_step = [&](int g) {
        const int cb = g / NSTEP, s = g - cb * NSTEP;
        const int tap = s >> 1, ch = s & 1;
        char* slot = ring + (g % NSLOT) * SLOT;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int piece = 2 * wave + k;
            int ll = lane;
            asm volatile("" : "+v"(ll));
            const int u = piece * 64 + ll, r = u >> 3, pc = u & 7;
            const int lc = pc ^ ((r >> 1) & 7);
            dma16(wrs, __builtin_amdgcn_readfirstlane(lds_addr(slot + piece * 1024)),
                  (((tap * NCO + cb) * CC + r) * CC + ch * 64 + lc * 8) * 2);
        }
    };

    int prev_b = -1;
    for (int tile = xcd_block(); tile < ntiles; tile += gridDim.x) {
        const int b = tile / tpi, rem = tile - b * tpi;
        const int r0 = (rem / tpr) * TR, w0 = (rem % tpr) * TW;
        issue_step(0);
        issue_step(1);
        issue_step(2);
        if (tid < CC) {
            if constexpr (MODE == 4) {
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) cst[cb * CC + tid] = A.bias[4 * tid + cb];   // packed row -> co = 4c + cb
            } else {
                cst[tid] = A.bias[tid];
            }
            if (MODE == 1 || MODE == 4) cst[4 * CC + tid] = A.alpha[tid];
        }
        // ---------------- the input image ----------------
        if constexpr (COMB) {
            // x_j = x_{j-1} + rs * s * t_{j-1} over the tile + halo: x and t chunks in flight while
            // the gate is computed.  The gate's operands (the image's tile sums, FC1, FC2) are
            // loaded FIRST: vmcnt retires in issue order, so gate operands issued behind the
            // 26 x / t chunks made the gate wait for the whole 198-KB staging before it could
            // start; issued ahead, the gate's reductions and FCs run while the staging lands
            constexpr int KU = (NUNIT + 511) / 512;   // 13
            const bool newimg = b != prev_b;
            // the gate's operands -- the image's tile sums (tpi x 512 B), FC1 and FC2 (Cr x 512 B
            // each) -- by LDS-DMA into the image area (free: the previous tile ended on a barrier),
            // ahead of the x / t chunks; the gate reads them from there
            // regions 1-KB aligned: a DMA piece writes whole KB (zeros past a region's end)
            const int sums_b = tpi * CC * 4, fc_b = A.Cr * CC * 4;
            const int o_w1 = (sums_b + 1023) & ~1023, o_w2 = o_w1 + ((fc_b + 1023) & ~1023);
#ifndef C128_GATE_REG
            const bool gate_lds = o_w2 + ((fc_b + 1023) & ~1023) <= IMG;
#else   // A/B only: the gate's operands through registers, issued behind the staging
            const bool gate_lds = false;
#endif
            const int c = tid & (CC - 1), g = tid >> 7;
            const int k1 = tid >> 4, j8 = (tid & 15) * 8;
            // FC2 lane layout: channel c2 = tid >> 2, hidden units k8 .. k8 + 7 (a quad per channel)
            const int c2 = tid >> 2, k8 = (tid & 3) * 8;
            if (newimg && gate_lds) {
                const i32x4 pr = make_rsrc(A.pp + (size_t)b * tpi * CC, (unsigned)sums_b);
                const i32x4 f1 = make_rsrc(A.pfc1, (unsigned)fc_b);
                const i32x4 f2 = make_rsrc(A.pfc2, (unsigned)fc_b);
                const int n0 = (sums_b + 1023) / 1024, n1 = (fc_b + 1023) / 1024;
                for (int piece = wave; piece < n0 + 2 * n1; piece += 8) {
                    int ll = lane;
                    asm volatile("" : "+v"(ll));
                    const bool s_ = piece < n0, a_ = !s_ && piece < n0 + n1;
                    const int loc = s_ ? piece : a_ ? piece - n0 : piece - n0 - n1;
                    char* dst = img + (s_ ? 0 : a_ ? o_w1 : o_w2) + loc * 1024;
                    dma16(s_ ? pr : a_ ? f1 : f2, __builtin_amdgcn_readfirstlane(lds_addr(dst)), (loc * 64 + ll) * 16);
                }
            }
            // the x / t chunks are the last KU * 2 vector-memory ops before the gate's wait
            asm volatile("" ::: "memory");
            const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, (int)act_bytes, 0x00020000);
            const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc((void*)A.tp, 0, (int)act_bytes, 0x00020000);
            uint4 xv[KU], tv[KU];
            unsigned offs[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) {
                const int u = tid + 512 * k;
                const int lrow = u / (ICOL * 16), rr = u - lrow * (ICOL * 16);
                const int col = rr >> 4, pc = rr & 15, lc = pc ^ (col & 15);
                const int gh = r0 - 1 + lrow, gw = w0 - 1 + col;
                const bool ok = u < NUNIT && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
                offs[k] = ok ? (unsigned)((((size_t)b * H + gh) * W + gw) * PXB + lc * 16) : OOB;
                xv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)offs[k], 0, 0));
                tv[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(trs, (int)offs[k], 0, 0));
            }
            asm volatile("" ::: "memory");
            if (newimg) {
                // the gate of image b (blocks.py:83-92): mean of t_{j-1} from its tile sums (fixed
                // order: tiles g, g + 4, ... per quarter, quarters in order), FC1 -> ReLU -> FC2 ->
                // sigmoid.  Waits for the gate operands only: the 2 KU x / t chunks stay in flight
                float w1[8], w2[8];
                {
                    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
                    if (gate_lds) {
                        asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
                        static_assert(2 * KU == 26, "the wait above counts the x / t chunks");
                        __syncthreads();                     // every wave's pieces landed
                        const float* pb = (const float*)img + c;
                        int k = g;
                        for (; k + 12 < tpi; k += 16) {
                            s0 += pb[k * CC];
                            s1 += pb[(k + 4) * CC];
                            s2 += pb[(k + 8) * CC];
                            s3 += pb[(k + 12) * CC];
                        }
                        for (; k < tpi; k += 4) s0 += pb[k * CC];
                        const float* w1p = (const float*)(img + o_w1) + (size_t)(k1 < A.Cr ? k1 : 0) * CC + j8;
                        const float* w2p = (const float*)(img + o_w2) + (size_t)c2 * A.Cr;
#pragma unroll
                        for (int e = 0; e < 8; ++e) w1[e] = k1 < A.Cr ? w1p[e] : 0.f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) w2[e] = k8 + e < A.Cr ? w2p[k8 + e] : 0.f;
                    } else {
                        const float* pb = A.pp + (size_t)b * tpi * CC + c;
                        int k = g;
                        for (; k + 12 < tpi; k += 16) {
                            s0 += pb[(size_t)k * CC];
                            s1 += pb[(size_t)(k + 4) * CC];
                            s2 += pb[(size_t)(k + 8) * CC];
                            s3 += pb[(size_t)(k + 12) * CC];
                        }
                        for (; k < tpi; k += 4) s0 += pb[(size_t)k * CC];
                        const float* w1p = A.pfc1 + (size_t)(k1 < A.Cr ? k1 : 0) * CC + j8;
#pragma unroll
                        for (int e = 0; e < 8; ++e) w1[e] = k1 < A.Cr ? w1p[e] : 0.f;
                        const float* w2p = A.pfc2 + (size_t)c2 * A.Cr;
#pragma unroll
                        for (int e = 0; e < 8; ++e) w2[e] = k8 + e < A.Cr ? w2p[k8 + e] : 0.f;
                    }
                    red[g * CC + c] = (s0 + s1) + (s2 + s3);
                }
                __syncthreads();
                if (tid < CC) scr[tid] = ((red[tid] + red[CC + tid]) + (red[2 * CC + tid] + red[3 * CC + tid])) * A.inv_hw;
                __syncthreads();
                {
                    // FC1 + ReLU: row k1 = tid >> 4 (k1 < Cr), 8 channels per lane, summed over the row of 16 lanes
                    float h = 0.f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) h += w1[e] * scr[j8 + e];
                    h = group16_sum(h);
                    if ((tid & 15) == 0) scr[CC + k1] = fmaxf(h, 0.f);
                }
                __syncthreads();
                {
                    float z = 0.f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) z += w2[e] * scr[CC + k8 + e];
                    z += dpp_f<0xB1>(z);                     // the quad's four partial sums
                    z += dpp_f<0x4E>(z);
                    if ((tid & 3) == 0) {
                        const float sg = 1.f / (1.f + expf(-z));
                        gate[c2] = sg * A.res_scale;
                        if (A.ps && rem == 0) A.ps[(size_t)b * CC + c2] = sg;
                    }
                }
                prev_b = b;
                __syncthreads();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            char* xo = (char*)A.xo;
#pragma unroll
            for (int k = 0; k < KU; ++k) {
                const int u = tid + 512 * k;
                if (u < NUNIT) {
                    const int lrow = u / (ICOL * 16), rr = u - lrow * (ICOL * 16);
                    const int col = rr >> 4, pc = rr & 15, lc = pc ^ (col & 15);
                    const float4 ga = *(const float4*)(gate + lc * 8);
                    const float4 gb = *(const float4*)(gate + lc * 8 + 4);
                    const float g8[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
                    float xf[8], tf[8], yv[8];
                    unpack16<T>(xv[k], xf);
                    unpack16<T>(tv[k], tf);
#pragma unroll
                    for (int e = 0; e < 8; ++e) yv[e] = tf[e] * g8[e] + xf[e];
                    const uint4 o = pack16<T>(yv);
                    *(uint4*)(img + u * 16) = o;
                    // the tile's own x_j (not the halo: its owner writes it) for the next RCAB
                    if (xo && lrow >= 1 && lrow <= TR && col >= 1 && col <= TW) *(uint4*)(xo + offs[k]) = o;
                }
            }
        } else {
            // plain input by LDS-DMA (zero padding: past-the-end offsets read 0)
            const i32x4 xr = make_rsrc(A.x, act_bytes);
            for (int k = 0; k < (NPIECE + 7) / 8; ++k) {
                const int piece = wave + 8 * k;
                if (piece >= NPIECE) break;
                int ll = lane;
                asm volatile("" : "+v"(ll));
                const int u = piece * 64 + ll;
                const int lrow = u / (ICOL * 16), rr = u - lrow * (ICOL * 16);
                const int col = rr >> 4, pc = rr & 15, lc = pc ^ (col & 15);
                const int gh = r0 - 1 + lrow, gw = w0 - 1 + col;
                const bool ok = (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
                const unsigned off = ok ? (unsigned)((((size_t)b * H + gh) * W + gw) * PXB + lc * 16) : OOB;
                dma16(xr, __builtin_amdgcn_readfirstlane(lds_addr(img + piece * 1024)), (int)off);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();   // the image, steps 0..2's filter slots and the constants visible

        // ---------------- the conv: NG filter steps (per 128-channel output block 9 taps x 2
        // input halves), each 2 k-halves of 16 MFMAs.  The barrier that publishes step g + 1's
        // slot sits between step g's two k-halves (their fragments already in registers), and the
        // same barrier frees step g's slot for the DMA of step g + 3: one barrier per step, its
        // wait hidden behind MFMAs.  Each k-half's fragments are re-read (for the next step) as
        // soon as its MFMAs are issued: 2 x 8 fragments live, no double buffer.
        uint4 A0[4], B0[4], A1[4], B1[4];
        auto load_half = [&](int g, int ks, uint4 (&a)[4], uint4 (&bv)[4]) {
            const int s = g % NSTEP;
            const int tap = s >> 1, ch = s & 1, kh = tap / 3, kw = tap - 3 * kh;
            const int bo = kw == 0 ? boffA : kw == 1 ? boffB : boffC;
            const char* ap = ring + (g % NSLOT) * SLOT + (aoff0 ^ (ks << 6));
            const char* bp = img + kh * IROW + (bo ^ ((4 * ks + 8 * ch) << 4));
#pragma unroll
            for (int m = 0; m < 4; ++m) a[m] = *(const uint4*)(ap + m * 2048);
#pragma unroll
            for (int p = 0; p < 4; ++p) bv[p] = *(const uint4*)(bp + p * 16 * PXB);
        };
        // publish step g + 1 (this wave's pieces landed; every wave's after the barrier) and
        // recycle step g's slot for step g + 3.  `extra`: epilogue stores issued after step
        // g + 1's DMA (mode 4's output block boundary)
        auto advance = [&](int g, int extra) {
            vm_wait((g + 2 < NG ? 2 : 0) + extra);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of step g done
            __syncthreads();
            if (g + 3 < NG) issue_step_fast(g + 3);
        };
        lane_offsets();
        load_half(0, 0, A0, B0);
        load_half(0, 1, A1, B1);
        f32x4 acc[4][4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[m][p] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int cb = 0; cb < NCO; ++cb) {
            for (int s = 0; s < NSTEP; ++s) {
                const int g = cb * NSTEP + s;
                const bool more = s < NSTEP - 1;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int p = 0; p < 4; ++p) mma16<T>(acc[m][p], A0[m], B0[p]);
                __builtin_amdgcn_sched_barrier(0);
                // a block's first step: the previous block's epilogue stores (8) went out after step
                // g + 1's DMA
                if (more) {
                    advance(g, (MODE == 4 && cb > 0 && s == 0) ? 8 : 0);
                    load_half(g + 1, 0, A0, B0);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int p = 0; p < 4; ++p) mma16<T>(acc[m][p], A1[m], B1[p]);
                __builtin_amdgcn_sched_barrier(0);
                if (more) load_half(g + 1, 1, A1, B1);
            }
            const int g = cb * NSTEP + NSTEP - 1;

            // ---------------- epilogue of output block cb: lane (q, c16) holds channels
            // 64 wh + 16 m + 4 q + i of pixel w0 + 16 p + c16 in row r0 + wr; pairs of m-blocks
            // become 16-B stores (pair16)
            const int q = lane >> 4, c16 = lane & 15;
            const size_t rowpx = ((size_t)b * H + r0 + wr) * W + w0 + c16;
            const int cho = 128 * wh + chunk_of(0, q) * 16;
            float tsum[4][4];                                   // mode 2: the row's channel sums
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int i = 0; i < 4; ++i) tsum[m][i] = 0.f;
#pragma unroll
            for (int mp = 0; mp < 2; ++mp) {
                float bia[2][4], alp[2][4];
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const int c0 = 64 * wh + 16 * (2 * mp + h2) + 4 * q;
                    const float4 bb4 = *(const float4*)(cst + (MODE == 4 ? cb * CC : 0) + c0);
                    bia[h2][0] = bb4.x, bia[h2][1] = bb4.y, bia[h2][2] = bb4.z, bia[h2][3] = bb4.w;
                    if constexpr (MODE == 1 || MODE == 4) {
                        const float4 aa4 = *(const float4*)(cst + 4 * CC + c0);
                        alp[h2][0] = aa4.x, alp[h2][1] = aa4.y, alp[h2][2] = aa4.z, alp[h2][3] = aa4.w;
                    }
                }
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    float v[2][4];
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[h2][i] = acc[2 * mp + h2][p][i] + bia[h2][i];
                    if constexpr (MODE == 1) {
                        if (A.z1) {
                            char* zb = (char*)A.z1 + (rowpx + 16 * p) * PXB + cho + mp * 64;
                            *(uint4*)zb = pair16(pk4<T>(v[0][0], v[0][1], v[0][2], v[0][3]),
                                                 pk4<T>(v[1][0], v[1][1], v[1][2], v[1][3]));
                        }
                    }
                    if constexpr (MODE == 2) {
#pragma unroll
                        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                            for (int i = 0; i < 4; ++i) tsum[2 * mp + h2][i] += v[h2][i];
                    }
                    if constexpr (MODE == 3) {
                        float rv[2][4];
#pragma unroll
                        for (int h2 = 0; h2 < 2; ++h2)
                            ld4<T>((const char*)A.res + (rowpx + 16 * p) * PXB + (64 * wh + 16 * (2 * mp + h2) + 4 * q) * 2,
                                   rv[h2]);
#pragma unroll
                        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                            for (int i = 0; i < 4; ++i) v[h2][i] += rv[h2][i];
                    }
                    if constexpr (MODE == 1 || MODE == 4) {
#pragma unroll
                        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                            for (int i = 0; i < 4; ++i) v[h2][i] = prelu_f(v[h2][i], alp[h2][i]);
                    }
                    const uint4 o = pair16(pk4<T>(v[0][0], v[0][1], v[0][2], v[0][3]),
                                           pk4<T>(v[1][0], v[1][1], v[1][2], v[1][3]));
                    if constexpr (MODE == 4) {
                        // conv block cb = sub-pixel (cb >> 1, cb & 1) of PixelShuffle(2), PReLU on
                        // the shuffled channel (custom.py's upsampler stage): out [B][2H][2W][128]
                        const size_t opx = ((size_t)b * 2 * H + 2 * (r0 + wr) + (cb >> 1)) * (2 * W) +
                                           2 * (w0 + 16 * p + c16) + (cb & 1);
                        *(uint4*)((char*)A.y + opx * PXB + cho + mp * 64) = o;
                    } else {
                        *(uint4*)((char*)A.y + (rowpx + 16 * p) * PXB + cho + mp * 64) = o;
                    }
                }
            }
            if constexpr (MODE == 2) {
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float sm = group16_sum(tsum[m][i]);
                        if (c16 == 0) red[wr * CC + 64 * wh + 16 * m + 4 * q + i] = sm;
                    }
            }
            if (g + 1 < NG) {
                // the next output block (mode 4): its first step's fragments; step g + 1's DMA is
                // older than this block's 8 stores
                advance(g, 8);
                load_half(g + 1, 0, A0, B0);
                load_half(g + 1, 1, A1, B1);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int p = 0; p < 4; ++p) acc[m][p] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }   // output blocks
        __syncthreads();   // the image and the ring are free for the next tile; red complete
        if constexpr (MODE == 2) {
            if (tid < CC)
                A.part[((size_t)b * tpi + rem) * CC + tid] =
                    (red[tid] + red[CC + tid]) + (red[2 * CC + tid] + red[3 * CC + tid]);
        }
    }
}

int g_c128_cus = 0;

template <typename T, int MODE, bool COMB>
void launch128(const K128& a, int grid, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_rcab128<T, MODE, COMB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS128);
        attr = true;
    }
    hipLaunchKernelGGL((k_rcab128<T, MODE, COMB>), dim3(grid), dim3(512), LDS128, s, a);
}

template <typename T>
void dispatch128(const K128& a, int mode, bool comb, int grid, hipStream_t s) {
    if (mode == 1) comb ? launch128<T, 1, true>(a, grid, s) : launch128<T, 1, false>(a, grid, s);
    else if (mode == 2) launch128<T, 2, false>(a, grid, s);
    else if (mode == 4) launch128<T, 4, false>(a, grid, s);
    else comb ? launch128<T, 3, true>(a, grid, s) : launch128<T, 3, false>(a, grid, s);
}

}  // namespace

extern "C" int fen_rcab_c128_supported(int dtype, int B, int H, int W, int C, int Cr) {
    if ((dtype != FEN_BF16 && dtype != FEN_F16) || C != CC || B <= 0 || H <= 0 || W <= 0 || H % TR || W % TW ||
        Cr <= 0 || Cr > 32)
        return 0;
    if ((size_t)B * H * W * PXB >= (size_t)0x7fff0000) return 0;      // 32-bit buffer offsets
    return 1;
}

extern "C" int fen_rcab_c128_tiles(int H, int W) { return (H / TR) * (W / TW); }

extern "C" int fen_rcab_c128(const fen_rcab_c128_desc* d, void* stream) {
    if (!d || !d->x || !d->w || !d->bias || !d->y) return FEN_EINVAL;
    if (!fen_rcab_c128_supported(d->dtype, d->B, d->H, d->W, d->C, d->Cr > 0 ? d->Cr : 1)) return FEN_EUNSUPPORTED;
    const int mode = d->mode;
    if (mode < 1 || mode > 4) return FEN_EINVAL;
    const bool comb = d->tp != nullptr;
    if (comb && (mode == 2 || mode == 4 || !d->pp || !d->pfc1 || !d->pfc2 || d->Cr <= 0 || d->Cr > 32)) return FEN_EINVAL;
    if ((mode == 1 || mode == 4) && !d->alpha) return FEN_EINVAL;
    if (mode == 4 && comb) return FEN_EINVAL;
    if (mode == 2 && !d->part) return FEN_EINVAL;
    if (mode == 3 && !d->res) return FEN_EINVAL;
    if (d->y == d->x || (comb && d->y == d->tp) || (d->xo && (d->xo == d->x || d->xo == d->tp))) return FEN_EINVAL;
    K128 a{};
    a.B = d->B, a.H = d->H, a.W = d->W, a.Cr = d->Cr;
    a.res_scale = d->res_scale, a.inv_hw = 1.0f / (float)(d->H * d->W);
    a.x = d->x, a.tp = d->tp, a.pp = d->pp, a.pfc1 = d->pfc1, a.pfc2 = d->pfc2, a.ps = d->ps;
    a.xo = comb ? d->xo : nullptr;
    a.w = d->w, a.bias = d->bias, a.alpha = d->alpha, a.res = d->res, a.y = d->y, a.z1 = d->z1, a.part = d->part;
    if (g_c128_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_c128_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_c128_cus <= 0) g_c128_cus = 256;
    }
    const int ntiles = d->B * (d->H / TR) * (d->W / TW);
    const int grid = ntiles < g_c128_cus ? ntiles : g_c128_cus;
    hipStream_t s = (hipStream_t)stream;
    if (d->dtype == FEN_F16) dispatch128<f16>(a, mode, comb, grid, s);
    else dispatch128<bf16>(a, mode, comb, grid, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

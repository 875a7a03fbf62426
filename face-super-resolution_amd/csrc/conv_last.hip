// conv_last as a persistent HBM-streaming kernel (bf16 / fp16, Cin = 64, Cout <= 4, x4 skip):
//   sr = conv3x3(a, w_last) + b_last + bicubic_x4(lr)          (custom.py:121-124, 158-161)
//   eval: clamp to [0, 1] (custom.py:181-188); training: |sr - hr| tile sums and the L1
//   gradient sign(sr - hr) * l1_scale in the NHWC16 layout the dgrad consumes.
//
// The op reads the 256x256x64 bf16 feature map once (268 MB at B = 32) and does 16x fewer
// MFMAs than an RCAB conv of the same size: it is HBM-bound, and what matters is keeping
// bytes in flight and no wave waiting on memory latency.  Structure (one 640-thread block
// per CU, persistent over 16x16 tiles):
//   * waves 8 and 9 are loaders: they alone issue every global read of a tile by LDS-DMA --
//     the 18x18 px halo (41 pieces, split between them), the 8x8 LR patch of each channel
//     (4-B DMA, border-clamped per element) and, in training, the 16x16 target pixels --
//     into a 3-slot ring two tiles ahead, and publish a tile with their own vmcnt + the
//     block barrier;
//   * waves 0..7 compute 2 output rows x 16 columns each (9 taps x 2 k-halves of 16x16x32
//     MFMAs, Cout padded to 16 rows, the halo-row-reuse order) and the epilogue, reading
//     only LDS: they issue no global loads, so none of them ever waits on memory (an
//     earlier form that loaded the LR patch itself waited ~2 us per tile on those loads,
//     which vmcnt also queues behind the previous tile's output stores);
//   * the bicubic skip: a horizontal then a vertical 4-tap pass over the patch, in the same
//     operation order as bicubic_sample (fen_common.h);
//   * the tile's loss sum is combined over the 8 waves through LDS and written one
//     iteration later (no extra barrier).
#include "fen_common.h"

namespace {

constexpr int NS = 3;                           // ring slots
constexpr int RPW = 2;                          // output rows per compute wave
constexpr int NCW = 16 / RPW;                   // compute waves (2 per SIMD: each hides its partner's latency)
constexpr int LW = NCW;                         // loader waves are LW, LW + 1
constexpr int CL_THREADS = 64 * (LW + 2);
constexpr int LR_P = 8;                         // LR patch: [4 ch][8 rows][8 cols] f32 = 1 KB
constexpr int O_W = NS * HALO_SLOT;             // 9 taps x [16 co][64 ci] bf16, swz rows
constexpr int W_BYTES = 9 * 16 * 128;
constexpr int O_LR = O_W + W_BYTES;             // NS x 1 KB
constexpr int O_HR = O_LR + NS * 1024;          // NS x [4 ch][16 rows][16 cols] f32 = 4 KB
constexpr int O_RED = O_HR + NS * 4096;         // [2][NCW] f32 per-wave loss sums
constexpr int CL_LDS = O_RED + 2 * NCW * 4;
constexpr int PIECES0 = (HALO_DMA + 1) / 2 + 4; // loader 0: even halo pieces + 4 LR pieces
constexpr int PIECES1 = HALO_DMA / 2;           // loader 1: odd halo pieces (+ 4 target pieces)
static_assert(CL_LDS <= 163840, "LDS budget");
static_assert(2 * PIECES0 <= 63 && 2 * (PIECES1 + 4) <= 63, "vmcnt field");

template <typename T, bool TRAIN>
__global__ __launch_bounds__(CL_THREADS, 1) void k_conv_last(const fen_conv_desc d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int q = lane >> 4, c16 = lane & 15;
    const int H = d.H, W = d.W, B = d.B, Cout = d.Cout;
    const int Hs = H >> 2, Ws = W >> 2;
    const int twn = W >> 4, tpi = twn * (H >> 4), ntiles = B * tpi;
    const int G = gridDim.x;
    const int slot = xcd_block();                     // neighbouring tiles on one XCD (shared halo rows)
    const int nmine = (ntiles - slot + G - 1) / G;
    constexpr bool train = TRAIN;
    float* red = (float*)(smem + O_RED);

    // weights -> LDS: packed [9][16][64] bf16, row = tap * 16 + co
    for (int i = tid; i < 9 * 16 * 8; i += CL_THREADS)
        *(uint4*)(smem + O_W + swz(i >> 3, i & 7)) = *(const uint4*)((const char*)d.w + (size_t)i * 16);
    __syncthreads();

    // ---- loaders: per-lane piece addressing, fixed for the launch (a single wave issues its
    //      pieces back to back, so the per-piece cost is an add for interior tiles)
    const int lw = wave - LW;                     // 0, 1 on the loader waves
    const i32x4 xr = make_rsrc(d.x, (unsigned)((size_t)B * H * W * 128));
    const i32x4 lrr = make_rsrc(d.lr, (unsigned)((size_t)B * Cout * Hs * Ws * 4));
    const i32x4 hrr = make_rsrc(train ? d.hr : d.lr, train ? (unsigned)((size_t)B * Cout * H * W * 4) : 0u);
    constexpr int PPW = (HALO_DMA + 1) / 2;
    int rel[PPW], hrc[PPW];
    if (lw >= 0) {
#pragma unroll
        for (int k = 0; k < PPW; ++k) {
            const int p = 2 * k + lw;
            const int s = p * 64 + lane, px = s >> 3, pc = s & 7;
            const int hr = px / HALO, hc = px - hr * HALO;
            rel[k] = (hr * W + hc) * 128 + ((pc ^ (hc & 7)) << 4);
            hrc[k] = px < HP ? (hr | (hc << 16)) : 0x7fff7fff;   // slack lanes: never in bounds
        }
    }
    auto issue = [&](int i) {                     // everything my i-th tile reads -> slot i % NS
        const int t = slot + i * G;
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const int sl = i % NS;
        const unsigned slot = lds_addr(smem + sl * HALO_SLOT);
        const int base = ((b * H + h0 - 1) * W + w0 - 1) * 128;
        if (h0 > 0 && w0 > 0 && h0 + 16 < H && w0 + 16 < W) {
#pragma unroll
            for (int k = 0; k < PPW; ++k) {
                const int p = 2 * k + lw;
                if (p >= HALO_DMA) break;
                const int voff = (2 * k + 2) * 8 <= HP ? base + rel[k] : (hrc[k] == 0x7fff7fff ? 0x7ffffff0 : base + rel[k]);
                dma16(xr, __builtin_amdgcn_readfirstlane(slot + p * 1024), voff);
            }
        } else {
#pragma unroll
            for (int k = 0; k < PPW; ++k) {
                const int p = 2 * k + lw;
                if (p >= HALO_DMA) break;
                const int gh = h0 - 1 + (hrc[k] & 0xffff), gw = w0 - 1 + (hrc[k] >> 16);
                const int voff = ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W) ? base + rel[k] : 0x7ffffff0;
                dma16(xr, __builtin_amdgcn_readfirstlane(slot + p * 1024), voff);
            }
        }
        if (lw == 0) {
            // LR patch rows h0/4-2.., cols w0/4-2.. of channel ch: lane = row * 8 + col
            const int gy = min(max((h0 >> 2) - 2 + (lane >> 3), 0), Hs - 1);
            const int gx = min(max((w0 >> 2) - 2 + (lane & 7), 0), Ws - 1);
            const unsigned lslot = lds_addr(smem + O_LR + sl * 1024);
#pragma unroll
            for (int ch = 0; ch < 4; ++ch) {
                const int voff = ch < Cout ? (((b * Cout + ch) * Hs + gy) * Ws + gx) * 4 : 0x7ffffff0;
                dma4(lrr, __builtin_amdgcn_readfirstlane(lslot + ch * 256), voff);
            }
        } else if (train) {
            // target rows h0.., 16 floats each: lane = row * 4 + 16-B chunk
            const unsigned hslot = lds_addr(smem + O_HR + sl * 4096);
#pragma unroll
            for (int ch = 0; ch < 4; ++ch) {
                const int voff = ch < Cout ? ((((b * Cout + ch) * H + h0 + (lane >> 2)) * W + w0) + (lane & 3) * 4) * 4
                                           : 0x7ffffff0;
                dma16(hrr, __builtin_amdgcn_readfirstlane(hslot + ch * 1024), voff);
            }
        }
    };
    if (lw >= 0) {
        issue(0);
        if (nmine > 1) issue(1);
    }
    // diagnostic builds only (tools/gpu_t4.sh): CL_DIAG_NOCOMPUTE times the load stream alone,
    // CL_DIAG_NOLOAD the compute waves alone (on the first two tiles' bytes)

    // ---- compute-wave constants
    // epilogue lane (q, c16) owns output channel q of pixel c16 (q < Cout valid)
    const bool chq = (lane >> 4) < Cout;
    const float bias_q = ((d.epi & FEN_EPI_BIAS) && chq) ? d.bias[lane >> 4] : 0.f;
    const float inv = 0.25f;
    // this lane's column taps (fixed per lane: w0 % 4 == 0); patch column of tap 0
    const float sx = ((float)c16 + 0.5f) * inv - 0.5f;   // relative to w0 / 4
    const float fx = floorf(sx);
    float cx[4];
    cubic_coeffs(sx - fx, cx);
    const int relc = (int)fx + 1;

#pragma unroll 1
    for (int i = 0; i < nmine; ++i) {
        if (lw >= 0) {                            // this tile landed (the next may stay in flight)
            if (i + 1 < nmine) {
                if (lw == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES0) : "memory");
                else if (train) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES1 + 4) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES1) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (lw >= 0) {
#ifndef CL_DIAG_NOLOAD
            if (i + 2 < nmine) issue(i + 2);
#endif
            continue;
        }
#ifdef CL_DIAG_NOCOMPUTE
        continue;
#endif
        const int t = slot + i * G;
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const int sl = i % NS;
        // the previous tile's loss sum (its 4 wave sums landed before this barrier)
        if (i > 0 && train && d.loss_part && tid == 0) {
            const float* rp = red + ((i - 1) & 1) * NCW;
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < NCW; ++w) s += rp[w];
            d.loss_part[t - G] = s;
        }
        // ---- MFMAs: acc[n] = D[co = 4q + r][pixel (h0 + RPW wave + n, w0 + c16)]
        const char* hs = smem + sl * HALO_SLOT;
        f32x4 acc[RPW];
#pragma unroll
        for (int n = 0; n < RPW; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int chunk = kk * 4 + q;
                const char* hb = hs + hcol(c16 + kw, chunk) + (wave * RPW) * (HALO * 128);
                uint4 Bf[RPW + 2], A[3];
#pragma unroll
                for (int n = 0; n < RPW + 2; ++n) Bf[n] = *(const uint4*)(hb + n * (HALO * 128));
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) A[kh] = *(const uint4*)(smem + O_W + swz((kh * 3 + kw) * 16 + c16, chunk));
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int n = 0; n < RPW; ++n) mma16<T>(acc[n], A[kh], Bf[n + kh]);
            }
        // ---- bicubic skip, lane (q, c16) evaluates channel q.  Output row h0 + m (m = RPW wave
        //      + n) = 4a + m%4 with a = h0/4 + m/4: taps at LR rows a-2..a+1 (m%4 < 2) or
        //      a-1..a+2, i.e. patch rows m/4 + (0..3) or m/4 + (1..4); horizontal pass first
        const int pr0 = (wave * RPW) >> 2;        // patch row of LR row a - 2
        const float* lrp = (const float*)(smem + O_LR + sl * 1024) + (q * LR_P + pr0) * LR_P + relc;
        const int ph = (wave * RPW) & 3;          // m % 4 of this wave's first row
        float hrow[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* row = lrp + (r + (ph >= 2 ? 1 : 0)) * LR_P;
            hrow[r] = row[0] * cx[0] + row[1] * cx[1] + row[2] * cx[2] + row[3] * cx[3];
        }
        const float* hrp = (const float*)(smem + O_HR + sl * 4096) + (wave * RPW) * 16 + c16;
        float lsum = 0.f;
#pragma unroll
        for (int n = 0; n < RPW; ++n) {
            const int h = h0 + wave * RPW + n;
            // sy = a + (m%4 + 0.5)/4 - 0.5: the same taps for both rows of a wave (RPW = 2,
            // m%4 in {0,1} or {2,3}), only the weights differ
            const float sy = ((float)(ph + n) + 0.5f) * inv - 0.5f;
            const float fy = floorf(sy);
            float cy[4];
            cubic_coeffs(sy - fy, cy);
            float bic = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) bic += hrow[k] * cy[k];
            // conv value of channel q: lane (0, c16) holds co 0..3 of pixel c16 (acc[n][r], co =
            // 4q + r); every lane takes its channel's from there -- one 48-lane store per row
            // instead of exec-masked 16-lane stores per channel
            float cq = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float t = __shfl(acc[n][r], c16, 64);
                cq = q == r ? t : cq;
            }
            float v = cq + bias_q + bic;
            if (d.clamp) v = fminf(fmaxf(v, 0.f), 1.f);
            if (d.y && chq) ((float*)d.y)[(((size_t)b * Cout + q) * H + h) * W + w0 + c16] = v;
            if (train) {
                const float diff = chq ? v - hrp[q * 256 + n * 16] : 0.f;
                lsum += fabsf(diff);
                const float sg = diff > 0.f ? d.l1_scale : (diff < 0.f ? -d.l1_scale : 0.f);
                // dL/dsr, NHWC16: lane (q, c16) writes channels 4q..4q+3 (only q = 0 nonzero)
                float g4[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t = __shfl(sg, r * 16 + c16, 64);
                    g4[r] = q == 0 ? t : 0.f;
                }
                if (d.dout) st4<T>((char*)d.dout + (((size_t)(b * H + h) * W + w0 + c16) * 16 + q * 4) * 2, g4);
            }
        }
        if (train && d.loss_part) {
            lsum = wave_sum(lsum);
            if (lane == 0) red[(i & 1) * NCW + wave] = lsum;
        }
    }
    // the last tile's loss sum
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (nmine > 0 && train && d.loss_part && tid == 0) {
        const float* rp = red + ((nmine - 1) & 1) * NCW;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NCW; ++w) s += rp[w];
        d.loss_part[slot + (nmine - 1) * G] = s;
    }
}

int g_cus = 0;

}  // namespace

namespace fen_detail {

bool conv_last_fast_ok(const fen_conv_desc* d) {
    return (d->dtype == FEN_BF16 || d->dtype == FEN_F16) && d->Cin == 64 && d->Cout <= 4 && d->scale == 4 && d->H % 16 == 0 &&
           d->W % 16 == 0 && d->H <= 8192 && d->W <= 8192 && d->debug == 0 &&
           (size_t)d->B * d->H * d->W * 128 < (size_t)0x7fff0000;
}

int launch_conv_last(const fen_conv_desc* d, hipStream_t s) {
    if (g_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus <= 0) g_cus = 256;
    }
    const int ntiles = d->B * (d->H >> 4) * (d->W >> 4);
    const int grid = ntiles < g_cus ? ntiles : g_cus;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_conv_last<bf16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, CL_LDS);
        (void)hipFuncSetAttribute((const void*)k_conv_last<bf16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, CL_LDS);
        (void)hipFuncSetAttribute((const void*)k_conv_last<f16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, CL_LDS);
        (void)hipFuncSetAttribute((const void*)k_conv_last<f16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, CL_LDS);
        attr_set = true;
    }
    if (d->dtype == FEN_F16) {
        if (d->hr) hipLaunchKernelGGL((k_conv_last<f16, true>), dim3(grid), dim3(CL_THREADS), CL_LDS, s, *d);
        else hipLaunchKernelGGL((k_conv_last<f16, false>), dim3(grid), dim3(CL_THREADS), CL_LDS, s, *d);
    } else {
        if (d->hr) hipLaunchKernelGGL((k_conv_last<bf16, true>), dim3(grid), dim3(CL_THREADS), CL_LDS, s, *d);
        else hipLaunchKernelGGL((k_conv_last<bf16, false>), dim3(grid), dim3(CL_THREADS), CL_LDS, s, *d);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

}  // namespace fen_detail

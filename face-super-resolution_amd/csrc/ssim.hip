// SSIM (reference src/losses/ssim_loss.py:44-98, SSIMLoss 174-226; the trainer's validation
// metric trainer.py:630-634): zero-padded depthwise 11x11 Gaussian (sigma 1.5, normalised,
// outer product of a 1-D window) over pred, target, pred^2, target^2, pred*target; the SSIM
// map ((2 mp mt + C1)(2 spt + C2)) / ((mp^2 + mt^2 + C1)(spp + stt + C2)); its sum per tile.
//
// With GRAD the same launch also produces d(sum S)/d(pred) in closed form: with
// a = dS/dmp, b = dS/dE[p^2], c = dS/dE[pt] per pixel (zero outside the image),
//   d(sum S)/dp(k) = (G * a)(k) + 2 p(k) (G * b)(k) + t(k) (G * c)(k)
// (G symmetric, same zero padding).  One block = one 32x32 tile of one image plane: inputs
// on the tile + 10 px (LDS), separable passes, the map terms on the tile + 5 px, their
// filtered combination on the tile.  No intermediate map touches HBM.  fp32 throughout.
#include "fen_common.h"

#include <type_traits>

namespace {

constexpr int SR = 5;       // window radius (window 11)
#ifndef SSIM_G2_WAVES
#define SSIM_G2_WAVES 4     // k_ssim_g2, 16-bit gradient: 4 waves per SIMD (<= 128 VGPRs, no spill; 38 KB of LDS)
#endif
constexpr int ST = 32;      // output tile
struct SsimWin {
    float g[2 * SR + 1];
};

inline int nblk(size_t n, int t = 256) { return (int)((n + t - 1) / t); }

// Horizontal pass over NCH column chunks of CW outputs: thread keeps the CW + 10 inputs of
// its chunk in registers and reads each LDS element once.  Packed fp32 (v_pk_fma_f32): the
// (p, t) and (p^2, t^2) sums two at a time, p t alone -- 3 FMA instructions per tap, not 5.
__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// G*a + 2 p G*b + t G*c with the contraction spelled out: the fused kernel and k_ssim_g2 round
// it identically whatever the surrounding code lets the compiler fuse
__device__ __forceinline__ float ssim_dcomb(f32x2 mab, float mc, float p, float t) {
    return __builtin_fmaf(t, mc, __builtin_fmaf(2.f * p, mab.y, mab.x));
}

template <int CW>
__device__ __forceinline__ void hrow(const SsimWin& win, const float* p, const float* t, float (&o)[5][CW]) {
    f32x2 pt[CW + 2 * SR], sq[CW + 2 * SR];
    float cr[CW + 2 * SR];
#pragma unroll
    for (int i = 0; i < CW + 2 * SR; ++i) {
        pt[i] = f32x2{p[i], t[i]};
        sq[i] = pt[i] * pt[i];
        cr[i] = pt[i].x * pt[i].y;
    }
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        f32x2 s01 = {0.f, 0.f}, s23 = {0.f, 0.f};
        float s4 = 0.f;
#pragma unroll
        for (int j = 0; j < 2 * SR + 1; ++j) {
            const f32x2 g2 = {win.g[j], win.g[j]};
            s01 = pfma(g2, pt[c + j], s01);
            s23 = pfma(g2, sq[c + j], s23);
            s4 = fmaf(win.g[j], cr[c + j], s4);
        }
        o[0][c] = s01.x; o[1][c] = s01.y; o[2][c] = s23.x; o[3][c] = s23.y; o[4][c] = s4;
    }
}

// CB > 1 (grad_mode 2, C <= CB): one block takes every channel of its tile in turn, keeps each
// channel's gradient tile in LDS and adds them to the NHWC16 buffer once at the end, 4 channels
// per 8-B (16-bit) / 16-B (fp32) read-modify-write per pixel, every thread 4 pixels, the reads
// issued before the last channel's passes; instead of C blocks each rewriting one 2-byte
// channel of every pixel row.
// MT: the type of the two-launch form's a / b / c maps (k_ssim<false> writes them when `maps`
// is given): fp16 for a 16-bit gradient (half the bytes of fp32; its 2^-11 relative rounding is
// 8x below the bf16 rounding of the sum the gradient lands in), fp32 for an fp32 gradient
template <bool GRAD, typename T, int CB, typename MT = float>
__global__ __launch_bounds__(256) void k_ssim(int B, int C, int H, int W, const float* __restrict__ pred,
                                              const float* __restrict__ target, const SsimWin win, float C1,
                                              float C2, float* __restrict__ part, void* __restrict__ grad,
                                              float grad_scale, int grad_mode, float* __restrict__ maps) {
    constexpr int E1 = GRAD ? ST + 2 * SR : ST;   // where the map (and a, b, c) is needed
    constexpr int E2 = E1 + 2 * SR;               // where the inputs are needed
    constexpr int O1 = GRAD ? SR : 0;             // tile offset inside E1
    constexpr int CW = GRAD ? 7 : 8;              // register block of the map passes (E1 = 6 or 4 of them)
    constexpr int NCH = E1 / CW;
    // the vertical pass's row block: without GRAD, 4 rows (32 x 8 = 256 items, one per thread;
    // 8 rows left half the block idle)
    constexpr int CWV = GRAD ? CW : 4, NCHV = E1 / CWV;
    constexpr int CW2 = 8, NCH2 = ST / CW2;       // horizontal gradient pass: 8-column chunks
    constexpr int RV = 4, NRV = ST / RV;          // vertical gradient pass: 4-row chunks (ST * NRV = 256 items)
    constexpr int PS = E2 + 1;
    constexpr bool LDSG = GRAD && CB > 1;         // the gradient tiles kept in LDS
    // sb: p, t on E2 x E2; after the first pass, a / b / c on E1 x E1 (3 E1 (E1+1) <= 2 E2 PS)
    // without GRAD the horizontal sums overwrite the staged inputs -- every item takes its input
    // window into registers before a barrier, then writes its sums (one item per thread:
    // E2 * NCH <= 256) -- 27.7 KB of LDS instead of 42 KB: with one channel per block (92 VGPRs)
    // 5 blocks per CU, was 3 (SSIM_NO_ALIAS: separate arrays, A/B)
#ifndef SSIM_NO_ALIAS
    constexpr bool ALIAS = !GRAD;
#else
    constexpr bool ALIAS = false;
#endif
    constexpr int NSB = 2 * E2 * PS, NHP = 5 * E2 * (E1 + 1);
    __shared__ float sbuf[ALIAS ? (NSB > NHP ? NSB : NHP) : NSB + NHP];
    float* sb = sbuf;
    float (*hp)[E2][E1 + 1] = (float (*)[E2][E1 + 1])(ALIAS ? sbuf : sbuf + NSB);   // horizontal sums (reused for a, b, c)
    __shared__ float dg[LDSG ? CB : 1][LDSG ? ST : 1][LDSG ? ST + 1 : 1];   // per channel d(sum S)/dp
    __shared__ float red[4];
    static_assert(3 * E1 * (E1 + 1) <= 2 * E2 * PS, "a/b/c alias");
    static_assert(ST * NRV == 256, "one vertical gradient item per thread");
    float* sp = sb;
    float* st = sb + E2 * PS;
    float (*abc)[E1][E1 + 1] = (float (*)[E1][E1 + 1])sb;
    const int tid = threadIdx.x;
    const int h0 = blockIdx.y * ST, w0 = blockIdx.x * ST;
    const int gy0 = h0 - O1 - SR, gx0 = w0 - O1 - SR;     // image coords of E2's (0, 0)
    const int b = CB > 1 ? (int)blockIdx.z : (int)blockIdx.z / C;
    // the E2 x E2 inputs of a channel: every load of the thread issued before the first LDS write
    // (one memory round trip per channel instead of one per 256 elements); with CB > 1 the next
    // channel's are issued as soon as this one's are in LDS, under its passes
    constexpr int NLD = (E2 * E2 + 255) / 256;
    float lp[NLD], lt[NLD];
    auto load_in = [&](int chn) {
        const size_t pl = (size_t)(b * C + chn) * H * W;
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int i = tid + k * 256;
            const int r = i / E2, c = i % E2, gy = gy0 + r, gx = gx0 + c;
            const bool in = i < E2 * E2 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
            const size_t e = in ? pl + (size_t)gy * W + gx : 0;
            lp[k] = in ? pred[e] : 0.f;
            lt[k] = in ? target[e] : 0.f;
        }
    };
    // the final read-modify-write's pixels: thread tid takes pixels tid + 256 k of the tile (row-
    // major: a wave's 64 lanes are two tile rows, 32 consecutive pixels each)
    typedef typename std::conditional<sizeof(T) == 2, uint2, float4>::type GV;
    GV gv[4];
    auto grad_ptr = [&](int k) -> GV* {
        const int pix = tid + 256 * k, gy = h0 + pix / ST, gx = w0 + pix % ST;
        return (gy < H && gx < W) ? (GV*)((T*)grad + (((size_t)b * H + gy) * W + gx) * 16) : nullptr;
    };
    load_in(CB > 1 ? 0 : (int)blockIdx.z % C);
#pragma unroll
    for (int cc = 0; cc < CB; ++cc) {
    if (CB > 1 && cc >= C) break;
    const int ch = CB > 1 ? cc : (int)blockIdx.z % C;
    const int plane = b * C + ch;
    const float* pp = pred + (size_t)plane * H * W;
    const float* tp = target + (size_t)plane * H * W;
    if (CB > 1 && cc > 0) __syncthreads();                // the previous channel's reads of sb / hp / red done
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
        const int i = tid + k * 256;
        if (i < E2 * E2) {
            const int r = i / E2, c = i % E2;
            sp[r * PS + c] = lp[k];
            st[r * PS + c] = lt[k];
        }
    }
    __syncthreads();
    if (CB > 1 && cc + 1 < CB && cc + 1 < C) load_in(cc + 1);
    if (LDSG && (cc + 1 == CB || cc + 1 == C)) {
        // the last channel: the gradient buffer's pixels in flight under its passes
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const GV* q = grad_ptr(k);
            if (q) gv[k] = *q;
        }
    }
    if constexpr (ALIAS) {
        static_assert(E2 * NCH <= 256, "one horizontal item per thread");
        const int r = tid / NCH, c0 = (tid % NCH) * CW;
        const bool item = tid < E2 * NCH;
        float pw[CW + 2 * SR], tw[CW + 2 * SR];
        if (item) {
#pragma unroll
            for (int k = 0; k < CW + 2 * SR; ++k) pw[k] = sp[r * PS + c0 + k], tw[k] = st[r * PS + c0 + k];
        }
        __syncthreads();                                    // every window in registers: sb is hp's now
        if (item) {
            float o[5][CW];
            hrow<CW>(win, pw, tw, o);
#pragma unroll
            for (int k = 0; k < 5; ++k)
#pragma unroll
                for (int c = 0; c < CW; ++c) hp[k][r][c0 + c] = o[k][c];
        }
    } else {
        for (int i = tid; i < E2 * NCH; i += 256) {
            const int r = i / NCH, c0 = (i % NCH) * CW;
            float o[5][CW];
            hrow<CW>(win, sp + r * PS + c0, st + r * PS + c0, o);
#pragma unroll
            for (int k = 0; k < 5; ++k)
#pragma unroll
                for (int c = 0; c < CW; ++c) hp[k][r][c0 + c] = o[k][c];
        }
    }
    __syncthreads();
    // vertical pass: thread = (column, CW-row chunk), the chunk's CW + 10 rows read once; the
    // (mp, mt) and (E[p^2], E[t^2]) sums packed
    float acc = 0.f;
    for (int i = tid; i < E1 * NCHV; i += 256) {
        const int c = i % E1, r0 = (i / E1) * CWV;
        f32x2 m01[CWV], m23[CWV];
        float m4[CWV];
#pragma unroll
        for (int o = 0; o < CWV; ++o) m01[o] = m23[o] = f32x2{0.f, 0.f}, m4[o] = 0.f;
#pragma unroll
        for (int rr = 0; rr < CWV + 2 * SR; ++rr) {
            const f32x2 v01 = {hp[0][r0 + rr][c], hp[1][r0 + rr][c]};
            const f32x2 v23 = {hp[2][r0 + rr][c], hp[3][r0 + rr][c]};
            const float v4 = hp[4][r0 + rr][c];
#pragma unroll
            for (int o = 0; o < CWV; ++o) {
                const int j = rr - o;
                if (j >= 0 && j <= 2 * SR) {
                    const f32x2 g2 = {win.g[j], win.g[j]};
                    m01[o] = pfma(g2, v01, m01[o]);
                    m23[o] = pfma(g2, v23, m23[o]);
                    m4[o] = fmaf(win.g[j], v4, m4[o]);
                }
            }
        }
#pragma unroll
        for (int o = 0; o < CWV; ++o) {
            const int r = r0 + o;
            const float mp = m01[o].x, mt = m01[o].y;
            const float spp = m23[o].x - mp * mp, stt = m23[o].y - mt * mt, spt = m4[o] - mp * mt;
            const float A1 = 2.f * mp * mt + C1, A2 = 2.f * spt + C2;
            const float B1 = mp * mp + mt * mt + C1, B2 = spp + stt + C2;
            // v_rcp_f32 (1 ulp) for the five quotients: B1, B2 >= C1, C2 > 0 (no zero / denormal
            // divisor); IEEE division sequences here were a quarter of the kernel's VALU issue
            const float r1 = __builtin_amdgcn_rcpf(B1), r2 = __builtin_amdgcn_rcpf(B2), iB = r1 * r2;
            const float S = (A1 * A2) * iB;
            const int gy = h0 - O1 + r, gx = w0 - O1 + c;
            const bool in = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
            const bool own = r >= O1 && r < O1 + ST && c >= O1 && c < O1 + ST;
            if (in && own) acc += S;
            if constexpr (GRAD) {
                abc[0][r][c] = in ? 2.f * mt * (A2 - A1) * iB - 2.f * mp * S * (r1 - r2) : 0.f;
                abc[1][r][c] = in ? -S * r2 : 0.f;
                abc[2][r][c] = in ? 2.f * A1 * iB : 0.f;
            } else if (maps && in) {
                // the two-launch form's first half: the same a, b, c of the tile's own pixels
                // to the maps (k_ssim_g2 filters them over the tile + halo)
                const size_t np = (size_t)B * C * H * W, e = (size_t)plane * H * W + (size_t)gy * W + gx;
                MT* mq = (MT*)maps;
                mq[e] = (MT)(2.f * mt * (A2 - A1) * iB - 2.f * mp * S * (r1 - r2));
                mq[np + e] = (MT)(-S * r2);
                mq[2 * np + e] = (MT)(2.f * A1 * iB);
            }
        }
    }
    if constexpr (GRAD) {
        __syncthreads();
        for (int i = tid; i < E1 * NCH2; i += 256) {          // horizontal pass of a, b (packed) and c
            const int r = i / NCH2, c0 = (i % NCH2) * CW2;
            f32x2 vab[CW2 + 2 * SR];
            float vc[CW2 + 2 * SR];
#pragma unroll
            for (int q = 0; q < CW2 + 2 * SR; ++q) vab[q] = f32x2{abc[0][r][c0 + q], abc[1][r][c0 + q]}, vc[q] = abc[2][r][c0 + q];
#pragma unroll
            for (int c = 0; c < CW2; ++c) {
                f32x2 sab = {0.f, 0.f};
                float sc = 0.f;
#pragma unroll
                for (int j = 0; j < 2 * SR + 1; ++j) {
                    sab = pfma(f32x2{win.g[j], win.g[j]}, vab[c + j], sab);
                    sc = fmaf(win.g[j], vc[c + j], sc);
                }
                hp[0][r][c0 + c] = sab.x;
                hp[1][r][c0 + c] = sab.y;
                hp[2][r][c0 + c] = sc;
            }
        }
        __syncthreads();
        {                                                     // vertical pass + the gradient: one item per thread
            const int c = tid % ST, r0 = (tid / ST) * RV, gx = w0 + c;
            float pr[RV], tr[RV];                             // L2-hot: this block staged them
#pragma unroll
            for (int o = 0; o < RV; ++o) {
                const int gy = min(h0 + r0 + o, H - 1);
                const bool in = gx < W;
                pr[o] = in ? pp[(size_t)gy * W + gx] : 0.f;
                tr[o] = in ? tp[(size_t)gy * W + gx] : 0.f;
            }
            f32x2 mab[RV];
            float mc[RV];
#pragma unroll
            for (int o = 0; o < RV; ++o) mab[o] = f32x2{0.f, 0.f}, mc[o] = 0.f;
#pragma unroll
            for (int rr = 0; rr < RV + 2 * SR; ++rr) {
                const f32x2 vab = {hp[0][r0 + rr][c], hp[1][r0 + rr][c]};
                const float vc = hp[2][r0 + rr][c];
#pragma unroll
                for (int o = 0; o < RV; ++o) {
                    const int j = rr - o;
                    if (j >= 0 && j <= 2 * SR) {
                        mab[o] = pfma(f32x2{win.g[j], win.g[j]}, vab, mab[o]);
                        mc[o] = fmaf(win.g[j], vc, mc[o]);
                    }
                }
            }
#pragma unroll
            for (int o = 0; o < RV; ++o) {
                float d = grad_scale * ssim_dcomb(mab[o], mc[o], pr[o], tr[o]);
                asm volatile("" : "+v"(d));                 // rounded as in k_ssim_g2
                const int gy = h0 + r0 + o;
                if constexpr (LDSG) {
                    dg[cc][r0 + o][c] = d;
                } else if (gx < W && gy < H) {
                    const size_t e = (size_t)gy * W + gx;
                    if (grad_mode == 1) {
                        ((float*)grad)[(size_t)plane * H * W + e] = d;
                    } else {
                        T* q = (T*)grad + (((size_t)b * H + gy) * W + gx) * 16 + ch;
                        *q = fromf<T>(tof<T>(*q) + d);
                    }
                }
            }
        }
    }
    // the tile's SSIM sum: wave sums (fixed tree), then the 4 waves in order
    acc = wave_sum(acc);
    if ((tid & 63) == 0) red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
        const int ntile = gridDim.x * gridDim.y;
        part[((size_t)ch * ntile + blockIdx.y * gridDim.x + blockIdx.x) * B + b] = ((red[0] + red[1]) + red[2]) + red[3];
    }
    }   // channels
    if constexpr (LDSG) {
#ifdef SSIM_NO_RMW
        // A/B only: the gradient's read-modify-write skipped (kept live by an improbable store)
        if (dg[0][tid & 31][tid >> 5] == 1234.5f) ((float*)grad)[tid] = tof<T>(((const T*)&gv[0])[0]);
        return;
#endif
        __syncthreads();                                      // every channel's dg tile written
        // channels 0..3 of each pixel in one read-modify-write (channels >= C written back as read)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            GV* q = grad_ptr(k);
            if (!q) continue;
            const int pix = tid + 256 * k, r = pix / ST, c = pix % ST;
            GV u = gv[k];
            T* v = (T*)&u;
#pragma unroll
            for (int kk = 0; kk < CB && kk < 4; ++kk)
                if (kk < C) v[kk] = fromf<T>(tof<T>(v[kk]) + dg[kk][r][c]);
            *q = u;
        }
    }
}

// The two-launch form's second half (grad_mode 2, C <= CB): per 32x32 tile, every channel in
// turn, a / b / c of the tile + 5 px read back from the maps written by k_ssim<false> (zero
// outside the image, as the fused kernel's), then the fused kernel's gradient passes unchanged
// (horizontal a, b packed + c; vertical; d = G*a + 2 p G*b + t G*c) and the NHWC16 read-modify-
// write of channels 0..3 once per pixel.  The maps are fp16 for a 16-bit gradient (37.5 MB
// written + read at B = 32, 3 x 256^2: the pair takes 97-98 us, 115 with fp32 maps), fp32 for
// an fp32 one.  The split trades them for the fused kernel's 10-px input halo: its map passes ran on 52 x 42 and 42 x 42 per 32 x 32
// tile (2.1x and 1.7x the tile), here on 42 x 32 and 32 x 32 -- the kernel was VALU-bound.
template <typename T, int CB, typename MT = typename std::conditional<sizeof(T) == 2, _Float16, float>::type>
__global__ __launch_bounds__(256, sizeof(T) == 2 ? SSIM_G2_WAVES : 3) void k_ssim_g2(int B, int C, int H, int W, const float* __restrict__ pred,
                                                 const float* __restrict__ target, const SsimWin win,
                                                 const float* __restrict__ maps, void* __restrict__ grad,
                                                 float grad_scale) {
    constexpr int E1 = ST + 2 * SR;                   // 42: the maps on the tile + halo
    constexpr int CW2 = 8, NCH2 = ST / CW2;
    constexpr int RV = 4, NRV = ST / RV;
    static_assert(ST * NRV == 256, "one vertical item per thread");
    // no gradient tile in LDS: each thread keeps its vertical item's pixels (4 rows of one column)
    // of every channel in registers and read-modify-writes exactly those (38 KB of LDS: 4 blocks
    // per CU, was 51 KB: 3)
    __shared__ float abc[3][E1][E1 + 1];
    __shared__ float hp[3][E1][ST + 1];
    const int tid = threadIdx.x;
    const int h0 = blockIdx.y * ST, w0 = blockIdx.x * ST;
    const int b = blockIdx.z;
    const size_t np = (size_t)B * C * H * W;
    constexpr int NLD = (E1 * E1 + 255) / 256;        // 7
    float la[NLD], lb[NLD], lc[NLD];
    auto load_maps = [&](int ch) {
        const size_t pl = (size_t)(b * C + ch) * H * W;
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int i = tid + k * 256;
            const int r = i / E1, c = i % E1, gy = h0 - SR + r, gx = w0 - SR + c;
            const bool in = i < E1 * E1 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
            const size_t e = in ? pl + (size_t)gy * W + gx : 0;
            const MT* mq = (const MT*)maps;
            const float va = (float)mq[e], vb = (float)mq[np + e], vc = (float)mq[2 * np + e];
            la[k] = in ? va : 0.f;
            lb[k] = in ? vb : 0.f;
            lc[k] = in ? vc : 0.f;
        }
    };
    typedef typename std::conditional<sizeof(T) == 2, uint2, float4>::type GV;
    // the thread's vertical item: column vc_, rows vr0 .. vr0 + RV - 1 of the tile
    const int vc_ = tid % ST, vr0 = (tid / ST) * RV, vgx = w0 + vc_;
    GV gv[RV];
    float dv[CB][RV];
    auto grad_ptr = [&](int o) -> GV* {
        const int gy = h0 + vr0 + o;
        return (gy < H && vgx < W) ? (GV*)((T*)grad + (((size_t)b * H + gy) * W + vgx) * 16) : nullptr;
    };
    load_maps(0);
#pragma unroll
    for (int cc = 0; cc < CB; ++cc) {
        if (cc >= C) break;
        const float* pp = pred + (size_t)(b * C + cc) * H * W;
        const float* tp = target + (size_t)(b * C + cc) * H * W;
        if (cc > 0) __syncthreads();                  // the previous channel's reads of abc / hp done
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int i = tid + k * 256;
            if (i < E1 * E1) {
                const int r = i / E1, c = i % E1;
                abc[0][r][c] = la[k];
                abc[1][r][c] = lb[k];
                abc[2][r][c] = lc[k];
            }
        }
        __syncthreads();
#ifndef SSIM_G2_LATE_PF
        if (cc + 1 < CB && cc + 1 < C) load_maps(cc + 1);
#endif
        if (cc + 1 == CB || cc + 1 == C) {
#pragma unroll
            for (int o = 0; o < RV; ++o) {
                const GV* q = grad_ptr(o);
                if (q) gv[o] = *q;
            }
        }
        for (int i = tid; i < E1 * NCH2; i += 256) {          // horizontal pass of a, b (packed) and c
            const int r = i / NCH2, c0 = (i % NCH2) * CW2;
            // a, b (packed), then c: one operand row live at a time (register peak)
            {
                f32x2 vab[CW2 + 2 * SR];
#pragma unroll
                for (int q = 0; q < CW2 + 2 * SR; ++q) vab[q] = f32x2{abc[0][r][c0 + q], abc[1][r][c0 + q]};
#pragma unroll
                for (int c = 0; c < CW2; ++c) {
                    f32x2 sab = {0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < 2 * SR + 1; ++j) sab = pfma(f32x2{win.g[j], win.g[j]}, vab[c + j], sab);
                    hp[0][r][c0 + c] = sab.x;
                    hp[1][r][c0 + c] = sab.y;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                float vc[CW2 + 2 * SR];
#pragma unroll
                for (int q = 0; q < CW2 + 2 * SR; ++q) vc[q] = abc[2][r][c0 + q];
#pragma unroll
                for (int c = 0; c < CW2; ++c) {
                    float sc = 0.f;
#pragma unroll
                    for (int j = 0; j < 2 * SR + 1; ++j) sc = fmaf(win.g[j], vc[c + j], sc);
                    hp[2][r][c0 + c] = sc;
                }
            }
        }
        // this channel's pred / target at the thread's 4 output pixels, for the gradient formula
        // after the vertical pass (issued behind the horizontal pass: its registers are free)
        float pr[RV], tr[RV];
#pragma unroll
        for (int o = 0; o < RV; ++o) {
            const int gy = min(h0 + vr0 + o, H - 1);
            const size_t e = vgx < W ? (size_t)gy * W + vgx : 0;
            pr[o] = pp[e];
            tr[o] = tp[e];
        }
#ifdef SSIM_G2_LATE_PF
        // the next channel's maps issued after the horizontal pass (its registers free), in
        // flight under the vertical pass
        if (cc + 1 < CB && cc + 1 < C) load_maps(cc + 1);
#endif
        __syncthreads();
        {                                                     // vertical pass + the gradient
            const int c = vc_, r0 = vr0;
            f32x2 mab[RV];
            float mc[RV];
#pragma unroll
            for (int o = 0; o < RV; ++o) mab[o] = f32x2{0.f, 0.f}, mc[o] = 0.f;
#pragma unroll
            for (int rr = 0; rr < RV + 2 * SR; ++rr) {
                const f32x2 vab = {hp[0][r0 + rr][c], hp[1][r0 + rr][c]};
                const float vc = hp[2][r0 + rr][c];
#pragma unroll
                for (int o = 0; o < RV; ++o) {
                    const int j = rr - o;
                    if (j >= 0 && j <= 2 * SR) {
                        mab[o] = pfma(f32x2{win.g[j], win.g[j]}, vab, mab[o]);
                        mc[o] = fmaf(win.g[j], vc, mc[o]);
                    }
                }
            }
#pragma unroll
            for (int o = 0; o < RV; ++o) {
                // the product rounded (opaque: not contracted into the final add, which the fused
                // kernel's LDS round trip rounds apart)
                float d = grad_scale * ssim_dcomb(mab[o], mc[o], pr[o], tr[o]);
                asm volatile("" : "+v"(d));
                dv[cc][o] = d;
            }
        }
    }
    // channels 0..3 of each of the thread's pixels in one read-modify-write (channels >= C
    // written back as read)
#pragma unroll
    for (int o = 0; o < RV; ++o) {
        GV* q = grad_ptr(o);
        if (!q) continue;
        GV u = gv[o];
        T* v = (T*)&u;
#pragma unroll
        for (int kk = 0; kk < CB && kk < 4; ++kk)
            if (kk < C) v[kk] = fromf<T>(tof<T>(v[kk]) + dv[kk][o]);
        *q = u;
    }
}

}  // namespace

#define STREAM ((hipStream_t)stream)

extern "C" size_t fen_ssim_parts(int B, int C, int H, int W) {
    return (size_t)C * ((H + ST - 1) / ST) * ((W + ST - 1) / ST);
}

extern "C" int fen_ssim(int dtype, int B, int C, int H, int W, const float* pred, const float* target,
                        const float* window1d, int window_size, float C1, float C2, float* part, void* grad,
                        float grad_scale, int grad_mode, void* stream) {
    if (!pred || !target || !window1d || !part || B <= 0 || C <= 0 || H <= 0 || W <= 0) return FEN_EINVAL;
    if (window_size != 2 * SR + 1) return FEN_EUNSUPPORTED;
    if (grad_mode < 0 || grad_mode > 2 || (grad_mode && !grad) || (grad_mode == 2 && C > 16)) return FEN_EINVAL;
    SsimWin w;
    for (int j = 0; j < 2 * SR + 1; ++j) w.g[j] = window1d[j];
    const dim3 grid((W + ST - 1) / ST, (H + ST - 1) / ST, B * C);
    const dim3 gridb((W + ST - 1) / ST, (H + ST - 1) / ST, B);      // CB: channels looped in the block
    if (grad_mode == 0 && C <= 3) {
        // one block per tile walks the channels, the next channel's inputs in flight under the
        // current one's passes
        hipLaunchKernelGGL((k_ssim<false, float, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                           C2, part, nullptr, 0.f, 0, nullptr);
    } else if (grad_mode == 0) {
        hipLaunchKernelGGL((k_ssim<false, float, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, nullptr, 0.f, 0, nullptr);
    } else if (grad_mode == 1) {
        hipLaunchKernelGGL((k_ssim<true, float, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode, nullptr);
    } else if (C <= 3 && (dtype == FEN_F32 || dtype == FEN_BF16)) {
        if (dtype == FEN_F32)
            hipLaunchKernelGGL((k_ssim<true, float, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                               C2, part, grad, grad_scale, grad_mode, nullptr);
        else
            hipLaunchKernelGGL((k_ssim<true, bf16, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                               C2, part, grad, grad_scale, grad_mode, nullptr);
    } else if (dtype == FEN_F32) {
        hipLaunchKernelGGL((k_ssim<true, float, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode, nullptr);
    } else if (dtype == FEN_BF16) {
        hipLaunchKernelGGL((k_ssim<true, bf16, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode, nullptr);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_ssim_work_floats(int B, int C, int H, int W) { return (size_t)3 * B * C * H * W; }

extern "C" int fen_ssim_ex(int dtype, int B, int C, int H, int W, const float* pred, const float* target,
                           const float* window1d, int window_size, float C1, float C2, float* part, void* grad,
                           float grad_scale, int grad_mode, float* work, void* stream) {
    const bool two = work && grad_mode == 2 && C <= 3 && (dtype == FEN_F32 || dtype == FEN_BF16);
    if (!two)
        return fen_ssim(dtype, B, C, H, W, pred, target, window1d, window_size, C1, C2, part, grad, grad_scale,
                        grad_mode, stream);
    if (!pred || !target || !window1d || !part || !grad || B <= 0 || H <= 0 || W <= 0) return FEN_EINVAL;
    if (window_size != 2 * SR + 1) return FEN_EUNSUPPORTED;
    SsimWin w;
    for (int j = 0; j < 2 * SR + 1; ++j) w.g[j] = window1d[j];
    const dim3 gridb((W + ST - 1) / ST, (H + ST - 1) / ST, B);
    // fp16 maps for a bf16 gradient only where a, b, c stay far inside fp16's range: |c| <= 2/C2,
    // |b| <= |S|/C2, |a| <= (2|mt| + 2|mp|)/C2 + 1/sqrt(C1) (B2 >= C2, A1 <= B1, |A2| <= B2); with
    // pixel values in [-1.5, 2.5] that is <= 8/C2 + 1/sqrt(C1).  Smaller constants than that
    // bound allows (the default C2 = 0.03^2 gives 8/C2 = 8.9e3) take fp32 maps: the same
    // gradient, 115 instead of 98 us at the bench shape (fen.h, fen_ssim_ex)
    const bool f16maps = dtype == FEN_BF16 && C1 > 0.f && C2 > 0.f && 8.f / C2 + 1.f / sqrtf(C1) <= 16384.f;
    // first half: the map, its tile sums and a / b / c (the fused kernel's non-gradient geometry)
#ifdef SSIM_EX_CB3   // A/B: one block per tile over the channels (3 blocks per CU)
    if (dtype == FEN_F32)
        hipLaunchKernelGGL((k_ssim<false, float, 3, float>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                           C2, part, nullptr, 0.f, 0, work);
    else
        hipLaunchKernelGGL((k_ssim<false, float, 3, _Float16>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w,
                           C1, C2, part, nullptr, 0.f, 0, work);
#else   // one block per (tile, channel): 5 blocks per CU (97-98 us for the pair vs 102-104)
    const dim3 gridc((W + ST - 1) / ST, (H + ST - 1) / ST, B * C);
    if (!f16maps)
        hipLaunchKernelGGL((k_ssim<false, float, 1, float>), gridc, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                           C2, part, nullptr, 0.f, 0, work);
    else
        hipLaunchKernelGGL((k_ssim<false, float, 1, _Float16>), gridc, dim3(256), 0, STREAM, B, C, H, W, pred, target, w,
                           C1, C2, part, nullptr, 0.f, 0, work);
#endif
    if (dtype == FEN_F32)
        hipLaunchKernelGGL((k_ssim_g2<float, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, work, grad,
                           grad_scale);
    else if (f16maps)
        hipLaunchKernelGGL((k_ssim_g2<bf16, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, work, grad,
                           grad_scale);
    else
        hipLaunchKernelGGL((k_ssim_g2<bf16, 3, float>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, work,
                           grad, grad_scale);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// Bandwidth-bound kernels of the FaceEnhanceNet hot path (gfx950): conv_first (K=27),
// conv_last data-gradient (K=27) fused with PReLU backward + PixelShuffle inverse, the
// channel-attention (SE) forward/backward pieces, the bicubic /4 LR synthesis, weight
// packing, deterministic column reductions and the fused clip_grad_norm_ + AdamW.
// All vector accesses are 16 B per lane.
#include "fen_common.h"
#include <type_traits>

namespace {

inline int nblk(size_t n, int t = 256) { return (int)((n + t - 1) / t); }

// ------------------------------ conv_first (3 -> C) ------------------------------
// reference custom.py:91-94,164; thread per (pixel, 8 output channels)
// (also the VGG19 input conv, perceptual.py:67-72,84-95: in-bounds samples normalised by
// (v - mean[ci]) * istd[ci] before the zero padding applies; and the discriminator's first
// block, discriminator.py:47-55: act >= 0 applies a leaky ReLU of slope act, ReLU = 0)
template <typename T>
__global__ void k_conv_first(int B, int Ci, int H, int W, int C, const float* __restrict__ x,
                             const float* __restrict__ w, const float* __restrict__ bias, T* __restrict__ y,
                             const float* __restrict__ in_mean, const float* __restrict__ in_istd, float act) {
    extern __shared__ __attribute__((aligned(16))) float sw[];  // [Ci*9][C]
    const int K = Ci * 9;
    for (int i = threadIdx.x; i < K * C; i += blockDim.x) {
        const int co = i % C, k = i / C;            // k = ci*9 + tap
        sw[i] = w[(size_t)co * K + k];
    }
    __syncthreads();
    const int G = C / 8;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)B * H * W * G) return;
    const int g = (int)(idx % G);
    const size_t px = idx / G;
    const int wq = (int)(px % W), hq = (int)((px / W) % H), b = (int)(px / ((size_t)W * H));
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bias[g * 8 + j];
    for (int ci = 0; ci < Ci; ++ci) {
        const float* xp = x + ((size_t)b * Ci + ci) * H * W;
        const float mu = in_mean ? in_mean[ci] : 0.f, is = in_istd ? in_istd[ci] : 1.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int hh = hq + t / 3 - 1, ww = wq + t % 3 - 1;
            const float v = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) ? (xp[(size_t)hh * W + ww] - mu) * is
                                                                                        : 0.f;
            const float4* wp = (const float4*)(sw + (ci * 9 + t) * C + g * 8);
            const float4 w0 = wp[0], w1 = wp[1];
            acc[0] += v * w0.x; acc[1] += v * w0.y; acc[2] += v * w0.z; acc[3] += v * w0.w;
            acc[4] += v * w1.x; acc[5] += v * w1.y; acc[6] += v * w1.z; acc[7] += v * w1.w;
        }
    }
    if (act >= 0.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = acc[j] > 0.f ? acc[j] : act * acc[j];
    }
    char* o = (char*)y + (px * C + g * 8) * sizeof(T);
    if constexpr (sizeof(T) == 2) {
        *(uint4*)o = pack16<T>(acc);
    } else {
        *(uint4*)o = pack16<float>(acc);
        *(uint4*)(o + 16) = pack16<float>(acc + 4);
    }
}

// The same conv, W % 4 == 0: a block computes a 2-row x 64-column output tile.  Its input
// halo (Ci x 4 x 66, zero-padded, normalised as above) is staged once in LDS with coalesced
// loads, and the filter with coalesced loads transposed into [k][co]; thread = (8 output
// channels, 4 consecutive pixels of a row) reads its 3 x 6 window per channel from LDS.  The
// one-pixel form above issued 27 global loads per thread, 8 lanes per pixel loading the same
// addresses: address-unit bound (~25 us at B = 32, 64x64).  Same per-output operation order
// (bias, then ci, then tap): bit-identical results.
constexpr int CF4_TW = 64;                      // tile width (output pixels)
template <typename T>
__global__ __launch_bounds__(256) void k_conv_first4(int B, int Ci, int H, int W, int C, const float* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     T* __restrict__ y, const float* __restrict__ in_mean,
                                                     const float* __restrict__ in_istd, float act) {
    extern __shared__ __attribute__((aligned(16))) float sw[];  // [Ci*9][C], then xs [Ci][4][CF4_TW + 2]
    constexpr int XR = CF4_TW + 2;
    const int K = Ci * 9;
    float* xs = sw + K * C;
    const int twn = (W + CF4_TW - 1) / CF4_TW, thn = (H + 1) >> 1;
    const int tile = blockIdx.x, b = tile / (thn * twn), r0 = ((tile / twn) % thn) * 2, c0 = (tile % twn) * CF4_TW;
    for (int i = threadIdx.x; i < K * C; i += blockDim.x) {     // w [co][k] read in order
        const int co = i / K, k = i - co * K;
        sw[k * C + co] = w[i];
    }
    for (int i = threadIdx.x; i < Ci * 4 * XR; i += blockDim.x) {
        const int ci = i / (4 * XR), rr = (i / XR) & 3, cc = i % XR;
        const int hh = r0 - 1 + rr, ww = c0 - 1 + cc;
        const float mu = in_mean ? in_mean[ci] : 0.f, is = in_istd ? in_istd[ci] : 1.f;
        xs[i] = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                    ? (x[(((size_t)b * Ci + ci) * H + hh) * W + ww] - mu) * is
                    : 0.f;
    }
    __syncthreads();
    const int G = C / 8;                          // channel groups; 256 / G threads cover the runs
    for (int tsk = threadIdx.x; tsk < G * 2 * (CF4_TW / 4); tsk += blockDim.x) {
        const int g = tsk % G, run = tsk / G;
        const int row = run / (CF4_TW / 4), cr = (run % (CF4_TW / 4)) * 4;
        const int hq = r0 + row, w0 = c0 + cr;
        if (hq >= H || w0 >= W) continue;
        float acc[4][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float bj = bias[g * 8 + j];
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[p][j] = bj;
        }
        for (int ci = 0; ci < Ci; ++ci) {
            float v[3][6];
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 6; ++c) v[r][c] = xs[(ci * 4 + row + r) * XR + cr + c];
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const float4* wp = (const float4*)(sw + (ci * 9 + t) * C + g * 8);
                const float4 wa = wp[0], wb = wp[1];
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const float vv = v[t / 3][p + t % 3];
                    acc[p][0] += vv * wa.x; acc[p][1] += vv * wa.y; acc[p][2] += vv * wa.z; acc[p][3] += vv * wa.w;
                    acc[p][4] += vv * wb.x; acc[p][5] += vv * wb.y; acc[p][6] += vv * wb.z; acc[p][7] += vv * wb.w;
                }
            }
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (act >= 0.f) {
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[p][j] = acc[p][j] > 0.f ? acc[p][j] : act * acc[p][j];
            }
            const size_t px = ((size_t)b * H + hq) * W + w0 + p;
            char* o = (char*)y + (px * C + g * 8) * sizeof(T);
            if constexpr (sizeof(T) == 2) {
                *(uint4*)o = pack16<T>(acc[p]);
            } else {
                *(uint4*)o = pack16<float>(acc[p]);
                *(uint4*)(o + 16) = pack16<float>(acc[p] + 4);
            }
        }
    }
}

// The same conv for 16-bit outputs on the f16 matrix cores: y^T[co][px] = W'[co][k] X[k][px]
// with K = 27 taps + a bias column (x = 1) padded to 32, one v_mfma_f32_16x16x32_f16 per
// (16 channels, 16 pixels).  fp32 accuracy is kept by splitting both operands into f16 hi + lo
// parts and summing hi*hi + hi*lo + lo*hi (the dropped lo*lo term is ~2^-22 relative), three
// MFMAs instead of 27 fp32 FMAs per output.  Blocks grid-stride over 16x16-pixel tiles: the
// normalised, zero-padded 3 x 18 x 18 halo is staged in LDS; wave w takes tile rows 4w..4w+3,
// lane = (pixel c16, k-slot group q).  The filter operand is built once per block in
// registers.  Each lane's accumulator holds 4 consecutive channels of one pixel; a wave stages
// its 16-pixel row in LDS and stores it as whole 16-byte lanes (the row is contiguous in NHWC),
// and the next tile's halo loads are in flight during the current tile's MFMAs.  The fp32 form above issued
// ~27 x 64 VALU FMAs per pixel (VALU bound at ~47 TFLOP/s on VGG conv1_1, 64 x 256^2).
constexpr int CFM16_BLOCKS = 2048;
template <typename T, int MB>
__global__ __launch_bounds__(256, MB <= 4 ? 5 : 1) void k_conv_first_m16(int B, int Ci, int H, int W, int C, const float* __restrict__ x,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       T* __restrict__ y, const float* __restrict__ in_mean,
                                                       const float* __restrict__ in_istd, float act) {
    __shared__ float xs[3 * 18 * 18];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int q = lane >> 4, c16 = lane & 15;
    const int th = (H + 15) >> 4, tw = (W + 15) >> 4;
    const int ntiles = B * th * tw, K = Ci * 9;
    // filter operand: lane holds W'[co = m*16 + c16][k = 8q + j], split hi / lo
    f16x8 ahi[MB], alo[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        const int co = m * 16 + c16;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * q + j;
            const float v = co < C ? (k < K ? w[(size_t)co * K + k] : (k == 27 ? bias[co] : 0.f)) : 0.f;
            const f16 h = (f16)v;
            ahi[m][j] = h;
            alo[m][j] = (f16)(v - (float)h);
        }
    }
    // activation operand: lane reads halo offset boff[j] (+ the pixel's), or the constant
    int boff[8];                                             // -1: the bias column (1), -2: padding (0)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * q + j;
        boff[j] = k < K ? (k / 9) * 324 + ((k % 9) / 3) * 18 + (k % 3) : (k == 27 ? -1 : -2);
    }
    // halo element i = tid + 256u: its channel is fixed per lane, so the normalisation is too;
    // loads are unconditional (clamped addresses, out-of-image elements zeroed at the LDS write)
    // so the prefetch stays in flight under the tile's MFMAs and stores
    __shared__ float nrm[2][3];                              // per-channel mean, 1/std
    if (tid < 3) {
        nrm[0][tid] = in_mean && tid < Ci ? in_mean[tid] : 0.f;
        nrm[1][tid] = in_istd && tid < Ci ? in_istd[tid] : 1.f;
    }
    float xv[4];
    unsigned inb = 0;
    auto load = [&](int t) {
        const int b = t / (th * tw), tt = t - b * th * tw;
        const int h0 = (tt / tw) << 4, w0 = (tt % tw) << 4;
        inb = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = min(tid + u * 256, 971);
            const int ci = i / 324, r = (i / 18) % 18, c = i % 18;
            const int hh = h0 - 1 + r, ww = w0 - 1 + c;
            if (ci < Ci && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) inb |= 1u << u;
            const int hc = min(max(hh, 0), H - 1), wc = min(max(ww, 0), W - 1);
            xv[u] = x[(((size_t)b * Ci + min(ci, Ci - 1)) * H + hc) * W + wc];
        }
    };
    constexpr int CC = MB * 16, PS = CC * 2 + 16;            // output staging: pixel stride (bytes)
    __shared__ __attribute__((aligned(16))) unsigned char ob[4][16 * PS];
    unsigned char* obw = ob[wave];
    if ((int)blockIdx.x < ntiles) load(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int b = t / (th * tw), tt = t - b * th * tw;
        const int h0 = (tt / tw) << 4, w0 = (tt % tw) << 4;
        __syncthreads();                                     // the previous tile's reads are done
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (tid + u * 256 < 972) {
                const int ci = (tid + u * 256) / 324;
                xs[tid + u * 256] = (inb >> u) & 1 ? (xv[u] - nrm[0][ci]) * nrm[1][ci] : 0.f;
            }
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);   // the next tile, in flight
        // ragged edges: rows past H and columns past W recompute the last valid row / column, and
        // their stores rewrite those bytes with the same values, so every wave issues the same
        // unconditional stores on every tile (the next halo's wait then skips them: vmcnt(8))
        const int nw = min(16, W - w0), rmax = H - 1 - h0;
        const int cc = min(c16, nw - 1);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int r = min(wave * 4 + g, rmax), hh = h0 + r;
            f16x8 bhi, blo;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = boff[j] >= 0 ? xs[boff[j] + r * 18 + cc] : (boff[j] == -1 ? 1.f : 0.f);
                const f16 h = (f16)v;
                bhi[j] = h;
                blo[j] = (f16)(v - (float)h);
            }
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[m], bhi, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[m], blo, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[m], bhi, acc, 0, 0, 0);
                // lane holds D[co = m*16 + 4q + e][px = c16]: staged as the row's NHWC image
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = act >= 0.f && acc[e] < 0.f ? act * acc[e] : acc[e];
                uint2 pk;
                pk.x = (unsigned)__builtin_bit_cast(unsigned short, (T)v[0]) |
                       ((unsigned)__builtin_bit_cast(unsigned short, (T)v[1]) << 16);
                pk.y = (unsigned)__builtin_bit_cast(unsigned short, (T)v[2]) |
                       ((unsigned)__builtin_bit_cast(unsigned short, (T)v[3]) << 16);
                *(uint2*)(obw + c16 * PS + (m * 16 + 4 * q) * 2) = pk;
            }
            // the row's outputs are contiguous in y (C = CC): 16-byte lanes, whole lines
            char* o = (char*)(y + (((size_t)b * H + hh) * W + w0) * CC);
            constexpr int CPP = CC / 8;                      // 16-byte chunks per pixel
#pragma unroll
            for (int s = 0; s < (16 * CPP + 63) / 64; ++s) {
                const int i = lane + 64 * s;
                if (16 * CPP >= 64 * (s + 1) || i < 16 * CPP) {
                    const int px = i / CPP, ch = i % CPP, pc = min(px, nw - 1);
                    *(uint4*)(o + (size_t)(pc * CPP + ch) * 16) = *(const uint4*)(obw + px * PS + ch * 16);
                }
            }
        }
    }
}

// conv_first weight gradient dw[co][ci][kh][kw] = sum_px dy[px][co] * x[ci][px + (kh-1, kw-1)]
// (+ db = sum_px dy).  Persistent blocks walk 16x16-pixel tiles in a fixed order (deterministic
// per-block partials): the tile's zero-padded 3 x 18 x 18 input halo is staged in LDS; wave w
// takes rows 4w..4w+3, lane = output channel (+64 for the second set); along a row the 3x3
// window of each input channel slides one column per pixel (9 LDS broadcast reads per pixel
// instead of 27 global loads) and the row's 16 dy values are loaded ahead.
constexpr int CF_BLOCKS = 512;
template <typename T>
__global__ __launch_bounds__(256) void k_conv_first_wgrad(int B, int Ci, int H, int W, int C, const float* __restrict__ x,
                                   const T* __restrict__ dy, float* __restrict__ part) {
    __shared__ float xs[3][18][19];
    __shared__ float red[4][28 * 2][64];
    const int lane = threadIdx.x & 63, wave = wave_id();
    const int nc = (C + 63) / 64;
    float acc[2][28];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int k = 0; k < 28; ++k) acc[j][k] = 0.f;
    const int th = (H + 15) >> 4, tw = (W + 15) >> 4;
    const int ntiles = B * th * tw;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int b = t / (th * tw), tt = t - b * th * tw;
        const int h0 = (tt / tw) << 4, w0 = (tt % tw) << 4;
        __syncthreads();                              // previous tile's window reads are done
        for (int i = threadIdx.x; i < 3 * 18 * 18; i += 256) {
            const int ci = i / 324, r = (i / 18) % 18, c = i % 18;
            const int hh = h0 - 1 + r, ww = w0 - 1 + c;
            xs[ci][r][c] = (ci < Ci && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                               ? x[(((size_t)b * Ci + ci) * H + hh) * W + ww] : 0.f;
        }
        __syncthreads();
#pragma unroll 1
        for (int rr = 0; rr < 4; ++rr) {
            const int r = wave * 4 + rr, hq = h0 + r;
            if (hq >= H) break;
            float g[2][16];
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const int wq = w0 + c;
                const size_t px = ((size_t)b * H + hq) * W + wq;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int co = lane + 64 * j;
                    g[j][c] = (j < nc && co < C && wq < W) ? tof<T>(dy[px * C + co]) : 0.f;
                }
            }
            float win[3][3][3];                       // [ci][kh][kw]
#pragma unroll
            for (int ci = 0; ci < 3; ++ci)
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    win[ci][kh][1] = xs[ci][r + kh][0];
                    win[ci][kh][2] = xs[ci][r + kh][1];
                }
#pragma unroll
            for (int c = 0; c < 16; ++c) {
#pragma unroll
                for (int ci = 0; ci < 3; ++ci)
#pragma unroll
                    for (int kh = 0; kh < 3; ++kh) {
                        win[ci][kh][0] = win[ci][kh][1];
                        win[ci][kh][1] = win[ci][kh][2];
                        win[ci][kh][2] = xs[ci][r + kh][c + 2];
                    }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (j >= nc) break;
#pragma unroll
                    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
                        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                            for (int kw = 0; kw < 3; ++kw) acc[j][ci * 9 + kh * 3 + kw] += g[j][c] * win[ci][kh][kw];
                    acc[j][27] += g[j][c];
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
        if (j < nc) {
#pragma unroll
            for (int k = 0; k < 28; ++k) red[wave][j * 28 + k][lane] = acc[j][k];
        }
    __syncthreads();
    for (int i = threadIdx.x; i < nc * 28 * 64; i += 256) {
        const int lanei = i & 63, jk = i >> 6;
        const float sum = red[0][jk][lanei] + red[1][jk][lanei] + red[2][jk][lanei] + red[3][jk][lanei];
        const int j = jk / 28, k = jk % 28, co = lanei + 64 * j;
        if (co < C) part[((size_t)blockIdx.x * 28 + k) * C + co] = sum;
    }
}

// The same weight gradient on the fp32 matrix cores: dW^T[co][k] = sum_px dy[px][co] X[px][k]
// with K = pixels, k = (ci, kh, kw) < 27 and k = 27 the bias column (X = 1), as
// v_mfma_f32_16x16x4_f32 (fp32 operands: the input image stays fp32, as in the VALU form).
// Persistent blocks walk 16x16-pixel tiles; per tile the 3 x 18 x 18 input halo and the
// 256 x C dy tile sit in LDS, each wave takes 4 pixel rows (16 k-steps of 4 pixels) for all
// C output channels (MB 16-row blocks) and both 16-column k blocks; the next tile's halo
// and dy are loaded into registers while the current one computes.  Each wave writes its own
// partial rows (4 per block), summed in fixed order by k_conv_first_finalize.
template <typename T, int MB>
__global__ __launch_bounds__(256) void k_conv_first_wgrad_m(int B, int Ci, int H, int W, int C,
                                                            const float* __restrict__ x, const T* __restrict__ dy,
                                                            float* __restrict__ part) {
    constexpr int CC = MB * 16;                              // channels held (C <= CC)
    constexpr int V = 16 / (int)sizeof(T);                   // dy elements per 16-B load
    constexpr int YV = 256 * CC / V / 256;                   // dy vectors per thread
    __shared__ float xs[3 * 18 * 18];
    __shared__ __attribute__((aligned(16))) T ys[256 * CC];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int q = lane >> 4, c16 = lane & 15;
    const int th = (H + 15) >> 4, tw = (W + 15) >> 4;
    const int ntiles = B * th * tw;
    // this lane's B-operand column k = nb * 16 + c16: halo offset (k < 27), bias (k = 27), 0
    int boff[2];
    float bconst[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        const int k = nb * 16 + c16;
        boff[nb] = k < 27 ? (k / 9) * 324 + ((k % 9) / 3) * 18 + (k % 3) : -1;
        bconst[nb] = k == 27 ? 1.f : 0.f;
    }
    f32x4 acc[MB][2];
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[m][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float xv[4];
    uint4 yv[YV];
    auto load = [&](int t) {
        const int b = t / (th * tw), tt = t - b * th * tw;
        const int h0 = (tt / tw) << 4, w0 = (tt % tw) << 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + u * 256;
            const int ci = i / 324, r = (i / 18) % 18, c = i % 18;
            const int hh = h0 - 1 + r, ww = w0 - 1 + c;
            xv[u] = (i < 972 && ci < Ci && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                        ? x[(((size_t)b * Ci + ci) * H + hh) * W + ww] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < YV; ++u) {
            const int i = tid + u * 256;                     // vector i: pixel i / (CC / V), chunk
            const int px = i / (CC / V), ch = i % (CC / V);
            const int hh = h0 + (px >> 4), ww = w0 + (px & 15);
            yv[u] = (hh < H && ww < W && ch * V < C)
                        ? *(const uint4*)(dy + (((size_t)b * H + hh) * W + ww) * C + ch * V) : make_uint4(0, 0, 0, 0);
        }
    };
    if ((int)blockIdx.x < ntiles) load(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        __syncthreads();                                     // the previous tile's reads are done
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (tid + u * 256 < 972) xs[tid + u * 256] = xv[u];
#pragma unroll
        for (int u = 0; u < YV; ++u) *(uint4*)(ys + (size_t)(tid + u * 256) * V) = yv[u];
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);   // the next tile, in flight
#pragma unroll 4
        for (int s = 0; s < 16; ++s) {
            const int px = wave * 64 + s * 4 + q, pr = px >> 4, pc = px & 15;
            float a[MB], bv[2];
#pragma unroll
            for (int m = 0; m < MB; ++m) a[m] = tof<T>(ys[px * CC + m * 16 + c16]);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) bv[nb] = boff[nb] >= 0 ? xs[boff[nb] + pr * 18 + pc] : bconst[nb];
#pragma unroll
            for (int m = 0; m < MB; ++m)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bv[nb], acc[m][nb], 0, 0, 0);
        }
    }
    // lane holds D[co = m*16 + 4q + r][k = nb*16 + c16]: the 4 waves' sums meet in LDS (over
    // ys, 448 * CC of its 512 * CC bytes) and the block writes one partial row set
    __syncthreads();
    float* red = (float*)ys;                                 // [wave][28][CC]
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = nb * 16 + c16, co = m * 16 + 4 * q + r;
                if (k < 28) red[(wave * 28 + k) * CC + co] = acc[m][nb][r];
            }
    __syncthreads();
    float* pb = part + (size_t)blockIdx.x * 28 * C;
    for (int i = tid; i < 28 * C; i += 256) {
        const int k = i / C, co = i - k * C;
        const float* rr = red + k * CC + co;
        pb[i] = (rr[0] + rr[28 * CC]) + (rr[56 * CC] + rr[84 * CC]);
    }
}

// block = one of the 28 rows k (27 weights + bias), 256 threads: thread (co, quarter) sums every
// 4th partial block (coalesced over co), fixed-order LDS combine -- deterministic
__global__ __launch_bounds__(1024) void k_conv_first_finalize(int nb, int Ci, int C, const float* part, float* dw,
                                                              float* db, int accum) {
    __shared__ float red[16][64];
    const int k = blockIdx.x;
    if (k >= Ci * 9 && k != 27) return;
    for (int c0 = 0; c0 < C; c0 += 64) {
        const int co = c0 + (threadIdx.x & 63), qr = threadIdx.x >> 6;
        float a = 0.f;
        if (co < C) {
#pragma unroll 8
            for (int r = qr; r < nb; r += 16) a += part[((size_t)r * 28 + k) * C + co];
        }
        red[qr][threadIdx.x & 63] = a;
        __syncthreads();
        if (threadIdx.x < 64 && co < C) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) s += red[j][threadIdx.x];
            if (k == 27) {
                if (db) db[co] = accum ? db[co] + s : s;
            } else {
                float* o = dw + (size_t)co * Ci * 9 + k;
                *o = accum ? *o + s : s;
            }
        }
        __syncthreads();
    }
}

// --------------- conv_last dgrad + PReLU backward + PixelShuffle inverse ---------------
// dout NHWC16 [B,H,W,16], w [Co][C][3][3] -> da[px][c] -> dv = da*(pre>0?1:alpha[c])
// -> du[b][h/2][w/2][4c + 2(h&1) + (w&1)];  block = 16x16 source px = 8x8 du px.
// Thread (k = tid % (C/2)) owns channels 2k, 2k+1 of du pixels tid / (C/2) + 256/(C/2) * j.
// The blocks stride over the tiles (grid = fen_conv_last_dgrad_part_rows, one slope-partial
// row each).
// Memory-latency bound (the FMAs are 7 GFLOP at B=32, 256x256): for 16-bit operands and
// C <= 64 (LPRE) the block's whole pre-activation tile (16x16 px x C, <= 32 KB) is loaded into
// LDS together with the dout halo -- one round trip per block instead of one per du pixel.
template <typename T, int C>
__global__ __launch_bounds__(256) void k_conv_last_dgrad(
                                  int B, int H, int W, int Co, const T* __restrict__ dout,
                                  const float* __restrict__ w, const T* __restrict__ pre, const T* __restrict__ post,
                                  const float* __restrict__ alpha, T* __restrict__ du, float* __restrict__ part) {
    constexpr int K2 = C / 2;
#ifdef CLD_GLOBAL_PRE   // A/B: the pre-activations read from global per du pixel
    constexpr bool LPRE = false;
#else
    constexpr bool LPRE = sizeof(T) == 2 && C <= 64;
#endif
    constexpr int PRE_U4 = LPRE ? 256 * C * 2 / 16 : 1;   // 16-B pieces of the tile
    __shared__ float4 sd[18 * 18];          // dout tile + halo, channels 0..2 (3 = pad)
    __shared__ float sdal[256 * 2];
    __shared__ uint4 spre[PRE_U4];          // [16 rows][16 px][C] pre-activations (LPRE)
    const int tid = threadIdx.x;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4), ntiles = B * tpi;
    const int k = tid % K2;                 // channel pair (2k, 2k+1), fixed per thread
    float wr[2][3][9];
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int co = 0; co < 3; ++co)
#pragma unroll
            for (int t = 0; t < 9; ++t)
                wr[e][co][t] = co < Co ? w[((size_t)co * C + 2 * k + e) * 9 + t] : 0.f;
    const float al0 = alpha[2 * k], al1 = alpha[2 * k + 1];
    // post (this pair's group of 4 has every slope > 0): p below is the PReLU output a, which has
    // the pre-activation's sign (all PReLU' needs); where a <= 0 the pre-activation is a / alpha,
    // so the slope gradient's sum of da * p * [p <= 0] is taken over a and scaled once at the end
    const bool rec = post && all_pos4(alpha + ((2 * k) & ~3));
    float dal0 = 0.f, dal1 = 0.f;
    const int Hh = H >> 1, Wh = W >> 1;
    // grid-stride over the tiles: one slope-partial row per block (fen_conv_last_dgrad_part_rows)
    for (int bt = blockIdx.x; bt < ntiles; bt += gridDim.x) {
    __syncthreads();                        // the previous tile's LDS reads done
    const int b = bt / tpi, tile = bt - b * tpi;
    const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
    if constexpr (LPRE) {
        constexpr int PPR = C * 2 / 16;     // 16-B pieces per pixel (8 channels: two groups of 4)
        static_assert(256 % PPR == 0, "a thread's pieces share one channel chunk");
        // each group of 4 channels from post (slopes all > 0: recovered below) or pre; the
        // thread's chunk (8 channels) is the same for all its pieces
        const int pcq = tid % PPR;
        // the tile is read from post when given (no wait on the slopes first); a half whose group
        // of 4 has a slope <= 0 is read again from pre afterwards (the rare case)
        const char* src = (const char*)(post ? post : pre);
        uint4 v[(PRE_U4 + 255) / 256];
#pragma unroll
        for (int j = 0; j < (PRE_U4 + 255) / 256; ++j) {
            const int i = tid + j * 256;
            const int px = i / PPR;
            const int gh = h0 + (px >> 4), gw = w0 + (px & 15);
            v[j] = make_uint4(0u, 0u, 0u, 0u);
            if (i < PRE_U4 && gh < H && gw < W)
                v[j] = *(const uint4*)(src + (((size_t)(b * H + gh) * W + gw) * C) * 2 + pcq * 16);
        }
        if (post) {
            const bool r0 = all_pos4(alpha + pcq * 8), r1 = all_pos4(alpha + pcq * 8 + 4);
            if (!(r0 && r1)) {
#pragma unroll
                for (int j = 0; j < (PRE_U4 + 255) / 256; ++j) {
                    const int i = tid + j * 256;
                    const int px = i / PPR;
                    const int gh = h0 + (px >> 4), gw = w0 + (px & 15);
                    if (i < PRE_U4 && gh < H && gw < W) {
                        const char* o = (const char*)pre + (((size_t)(b * H + gh) * W + gw) * C) * 2 + pcq * 16;
                        if (!r0) {
                            const uint2 lo = *(const uint2*)o;
                            v[j].x = lo.x, v[j].y = lo.y;
                        }
                        if (!r1) {
                            const uint2 hi = *(const uint2*)(o + 8);
                            v[j].z = hi.x, v[j].w = hi.y;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < (PRE_U4 + 255) / 256; ++j)
            if (tid + j * 256 < PRE_U4) spre[tid + j * 256] = v[j];
    }
    for (int i = tid; i < 18 * 18; i += 256) {
        const int r = i / 18, c = i % 18;
        const int gh = h0 + r - 1, gw = w0 + c - 1;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W) {
            float t4[4];
            ld4<T>((const char*)dout + ((size_t)(b * H + gh) * W + gw) * 16 * sizeof(T), t4);
            v = make_float4(t4[0], Co > 1 ? t4[1] : 0.f, Co > 2 ? t4[2] : 0.f, 0.f);
        }
        sd[i] = v;
    }
    __syncthreads();
    for (int i = tid; i < 64 * K2; i += 256) {
        const int dp = i / K2;
        const int hh = dp >> 3, ww = dp & 7;
        const int gh2 = (h0 >> 1) + hh, gw2 = (w0 >> 1) + ww;
        if (gh2 >= Hh || gw2 >= Wh) continue;
        float out[8];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int sh = 2 * hh + (t >> 1), sw = 2 * ww + (t & 1);   // local source pixel
            float da0 = 0.f, da1 = 0.f;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const float4 g = sd[(sh - kh + 2) * 18 + (sw - kw + 2)];
                    const int tp = kh * 3 + kw;
                    da0 += g.x * wr[0][0][tp] + g.y * wr[0][1][tp] + g.z * wr[0][2][tp];
                    da1 += g.x * wr[1][0][tp] + g.y * wr[1][1][tp] + g.z * wr[1][2][tp];
                }
            float p0, p1;
            if constexpr (LPRE) {
                const unsigned pw = ((const unsigned*)spre)[(sh * 16 + sw) * K2 + k];
                p0 = lo16<T>(pw);
                p1 = hi16<T>(pw);
            } else {
                const size_t pi = ((size_t)(b * H + h0 + sh) * W + w0 + sw) * C + 2 * k;
                const T* src = rec ? post : pre;
                p0 = tof<T>(src[pi]);
                p1 = tof<T>(src[pi + 1]);
            }
            dal0 += prelu_dalpha_f(da0, p0);
            dal1 += prelu_dalpha_f(da1, p1);
            out[t] = prelu_bwd_f(da0, p0, al0);
            out[4 + t] = prelu_bwd_f(da1, p1, al1);
        }
        char* o = (char*)du + (((size_t)(b * Hh + gh2) * Wh + gw2) * (4 * C) + 8 * k) * sizeof(T);
        if constexpr (sizeof(T) == 2) {
            *(uint4*)o = pack16<T>(out);
        } else {
            *(uint4*)o = pack16<float>(out);
            *(uint4*)(o + 16) = pack16<float>(out + 4);
        }
    }
    }
    if (rec) {
        dal0 *= __builtin_amdgcn_rcpf(al0);
        dal1 *= __builtin_amdgcn_rcpf(al1);
    }
    sdal[tid * 2] = dal0;
    sdal[tid * 2 + 1] = dal1;
    __syncthreads();
    if (tid < C) {
        const int kk = tid >> 1, e = tid & 1;
        float s = 0.f;
        for (int r = kk; r < 256; r += K2) s += sdal[r * 2 + e];
        part[(size_t)blockIdx.x * C + tid] = s;
    }
}

// The same for 16-bit operands and C = 64 (the network's last upsampler stage), persistent and
// pipelined: CLD_GRID blocks (two per CU) walk the tiles in order; while a block computes tile i
// from LDS its threads already hold tile i + 1's pre-activation chunks and dout halo in
// registers (one memory round trip per tile overlapped with the previous tile's FMAs instead of
// one exposed per block); the channel pair's two outputs as packed fp32 FMAs; the slope partials
// accumulate over the block's tiles (one partial row per block).  Same arithmetic per output as
// k_conv_last_dgrad (the same tap order), so the two agree to the summation order of dalpha.
constexpr int CLD_GRID = 512;
template <typename T>
__global__ __launch_bounds__(256, 2) void k_cld_p(int B, int H, int W, int Co, const T* __restrict__ dout,
                                                  const float* __restrict__ w, const T* __restrict__ pre,
                                                  const T* __restrict__ post, const float* __restrict__ alpha,
                                                  T* __restrict__ du, float* __restrict__ part) {
    constexpr int C = 64, K2 = 32, NV = 8;          // 8 x 16-B pieces of the 16x16x64 tile per thread
    __shared__ float4 sd[18 * 18];
    __shared__ uint4 spre[256 * 8];
    __shared__ float sdal[512];
    const int tid = threadIdx.x;
    const int twn = W >> 4, tpi = twn * (H >> 4), ntiles = B * tpi;
    const int pcq = tid & 7;                        // the thread's 8-channel chunk of every pixel it loads
    // each half (4 channels) of the chunk from post where the group's slopes are all > 0 (the
    // PReLU output has the pre-activation's sign), else from pre
    const bool plo = post && all_pos4(alpha + pcq * 8), phi = post && all_pos4(alpha + pcq * 8 + 4);
    const char* slo = (const char*)(plo ? post : pre);
    const char* shi = (const char*)(phi ? post : pre);
    uint4 pv[NV];
    uint2 dv[2];
    auto load = [&](int t) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int px = (tid >> 3) + 32 * j;
            const size_t o = (((size_t)(b * H + h0 + (px >> 4)) * W + w0 + (px & 15)) * C) * 2 + pcq * 16;
            if (slo == shi) {
                pv[j] = *(const uint4*)(slo + o);
            } else {
                const uint2 lo = *(const uint2*)(slo + o), hi = *(const uint2*)(shi + o + 8);
                pv[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + 256 * j, r = i / 18, c = i % 18;
            const int gh = h0 + r - 1, gw = w0 + c - 1;
            const bool in = i < 18 * 18 && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
            dv[j] = in ? *(const uint2*)((const char*)dout + ((size_t)(b * H + gh) * W + gw) * 16 * sizeof(T))
                       : make_uint2(0u, 0u);
        }
    };
    const int k = tid % K2;                         // channel pair (2k, 2k+1), fixed per thread
    f32x2 wr[3][9];
#pragma unroll
    for (int co = 0; co < 3; ++co)
#pragma unroll
        for (int tp = 0; tp < 9; ++tp)
            wr[co][tp] = co < Co ? f32x2{w[((size_t)co * C + 2 * k) * 9 + tp], w[((size_t)co * C + 2 * k + 1) * 9 + tp]}
                                 : f32x2{0.f, 0.f};
    const float al0 = alpha[2 * k], al1 = alpha[2 * k + 1];
    const bool rec = post && all_pos4(alpha + ((2 * k) & ~3));
    const int Hh = H >> 1, Wh = W >> 1;
    float dal0 = 0.f, dal1 = 0.f;
    int t = blockIdx.x;
    if (t < ntiles) load(t);
    for (; t < ntiles; t += gridDim.x) {
        __syncthreads();                            // the previous tile's LDS reads done
#pragma unroll
        for (int j = 0; j < NV; ++j) spre[tid + 256 * j] = pv[j];   // piece (px, pcq) at px * 8 + pcq
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + 256 * j;
            if (i < 18 * 18) {
                float t4[4];
                ld4<T>(&dv[j], t4);
                sd[i] = make_float4(t4[0], Co > 1 ? t4[1] : 0.f, Co > 2 ? t4[2] : 0.f, 0.f);
            }
        }
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);   // the next tile, in flight under the FMAs
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
#pragma unroll 2
        for (int m = 0; m < 8; ++m) {
            const int dp = (tid >> 5) + 8 * m;      // du pixel of the tile (8 x 8)
            const int hh = dp >> 3, ww = dp & 7;
            float out[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int sh = 2 * hh + (q >> 1), sw = 2 * ww + (q & 1);   // local source pixel
                f32x2 da = {0.f, 0.f};
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        const float4 g = sd[(sh - kh + 2) * 18 + (sw - kw + 2)];
                        const int tp = kh * 3 + kw;
                        da = __builtin_elementwise_fma(f32x2{g.x, g.x}, wr[0][tp], da);
                        da = __builtin_elementwise_fma(f32x2{g.y, g.y}, wr[1][tp], da);
                        da = __builtin_elementwise_fma(f32x2{g.z, g.z}, wr[2][tp], da);
                    }
                const unsigned pw = ((const unsigned*)spre)[(sh * 16 + sw) * K2 + k];
                const float p0 = lo16<T>(pw), p1 = hi16<T>(pw);
                dal0 += prelu_dalpha_f(da.x, p0);
                dal1 += prelu_dalpha_f(da.y, p1);
                out[q] = prelu_bwd_f(da.x, p0, al0);
                out[4 + q] = prelu_bwd_f(da.y, p1, al1);
            }
            *(uint4*)((char*)du + (((size_t)(b * Hh + (h0 >> 1) + hh) * Wh + (w0 >> 1) + ww) * (4 * C) + 8 * k) * sizeof(T)) =
                pack16<T>(out);
        }
    }
    if (rec) {
        dal0 *= __builtin_amdgcn_rcpf(al0);
        dal1 *= __builtin_amdgcn_rcpf(al1);
    }
    sdal[tid * 2] = dal0;
    sdal[tid * 2 + 1] = dal1;
    __syncthreads();
    if (tid < C) {
        const int kk = tid >> 1, e = tid & 1;
        float sum = 0.f;
        for (int r = kk; r < 256; r += K2) sum += sdal[r * 2 + e];
        part[(size_t)blockIdx.x * C + tid] = sum;
    }
}

// conv_last's whole backward in one pass (16-bit, C = 64, post given, whole 16x16 tiles):
//   du = unshuffle(PReLU'(conv_last^T dout)), the slope partials, and conv_last's weight and
//   bias gradients -- instead of k_conv_last_dgrad plus a separate weight-gradient pass that
//   reads the 268 MB stage output a second time (custom.py:177-184 backward).
// Both products are GEMMs over one im2col matrix of the dout halo, X[r][k] (r = the tile's 256
// source pixels, k = co * 9 + tap, 27 used of 32):
//   da[r][c]  = sum_k X[r][k] W[k][c]        (M = r, N = c, K = k; W split hi + lo in 16 bits,
//                                              two MFMAs: the fp32 weights to ~16 mantissa bits)
//   dW[k][c] += sum_r X[r][k] a[r][c]        (M = k, N = c, K = r; accumulated over the tiles)
// on 16x16x32 MFMAs.  Row order r = 4 * dp + q (dp = du pixel of the 8x8 du tile, q = 2 (h & 1) +
// (w & 1)): a lane's 4 accumulator rows are the 4 source pixels of one du pixel, i.e. the 4
// consecutive du channels 4c..4c+3 -- one 8-B store, 16 lanes 128 contiguous bytes.  LDS holds
// X (r-major, the dgrad's A), X^T and the activation tile P^T (c-major: the weight gradient's
// operands and the epilogue's 4 pixels of one channel in one 8-B read).  Persistent: CLD_GRID
// blocks walk the tiles, the next tile's activation pieces and dout halo in registers under the
// current tile's MFMAs; one partial row per block for the slopes, the weights and the bias.
// P holds post (a) for groups of 4 channels whose slopes are all > 0 (the pre-activation's sign,
// recovered as in k_conv_last_dgrad) and pre (v) for the others; the weight gradient needs a,
// rebuilt there as rnd16(PReLU(v)) (the forward rounded PReLU(acc) once: one rounding apart).
constexpr int CLB_XS = 40, CLB_TS = 264;   // 16-bit row strides of X, and of X^T / P^T (16-B aligned)
constexpr int CLB_LDS = 18 * 18 * 8 + 256 * CLB_XS * 2 + 32 * CLB_TS * 2 + 64 * CLB_TS * 2;
template <typename T>
__global__ __launch_bounds__(256, 2) void k_cl_bwd(int B, int H, int W, int Co, const T* __restrict__ dout,
                                                   const float* __restrict__ w, const T* __restrict__ pre,
                                                   const T* __restrict__ post, const float* __restrict__ alpha,
                                                   T* __restrict__ du, float* __restrict__ dal_part,
                                                   float* __restrict__ dw_part, float* __restrict__ db_part) {
    constexpr int C = 64, XS = CLB_XS, TS = CLB_TS;
    __shared__ __attribute__((aligned(16))) char smem[CLB_LDS];
    uint2* hd = (uint2*)smem;                                        // dout halo, channels 0..3
    unsigned short* X = (unsigned short*)(smem + 18 * 18 * 8);       // [256 r][XS]
    unsigned short* XT = X + 256 * XS;                               // [32 k][TS]
    unsigned short* PT = XT + 32 * TS;                               // [64 c][TS], 8-element chunks swizzled
    // P^T element (c, r): the 16-B chunk r >> 3 of row c XOR (c >> 3) & 7.  The transposed
    // writes (32 lanes of one ds_write_b32: 8 channel rows 8 apart x 4 pixel pairs) then fall on
    // 16 banks instead of 4 (every row of a channel group hit the same one: 8-way); the reads
    // (16 B at r % 8 == 0, 8 B at r % 4 == 0) stay inside one chunk
#ifndef CLB_NOSWZ
    auto pt = [&](int c, int r) { return PT + c * TS + (((r >> 3) ^ ((c >> 3) & 7)) << 3) + (r & 7); };
#else   // A/B only: the unswizzled layout
    auto pt = [&](int c, int r) { return PT + c * TS + r; };
#endif
    const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lq = lane >> 4;
    const int wave = wave_id();
    const int twn = W >> 4, tpi = twn * (H >> 4), ntiles = B * tpi;
    // ---- loads: 4 pixel pairs (2P, 2P + 1) x one 8-channel chunk per thread, + 2 halo pixels
    const int pcq = tid & 7, pp = tid >> 3;
    const bool plo = all_pos4(alpha + pcq * 8), phi = all_pos4(alpha + pcq * 8 + 4);
    const char* slo = (const char*)(plo ? post : pre);
    const char* shi = (const char*)(phi ? post : pre);
    uint4 pv[4][2];
    uint2 dv[2];
    auto load = [&](int t) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int px = 2 * (pp + 32 * j) + e;
                const size_t o = (((size_t)(b * H + h0 + (px >> 4)) * W + w0 + (px & 15)) * C) * 2 + pcq * 16;
                if (slo == shi) {
                    pv[j][e] = *(const uint4*)(slo + o);
                } else {
                    const uint2 lo = *(const uint2*)(slo + o), hi = *(const uint2*)(shi + o + 8);
                    pv[j][e] = make_uint4(lo.x, lo.y, hi.x, hi.y);
                }
            }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + 256 * j, r = i / 18, c = i % 18;
            const int gh = h0 + r - 1, gw = w0 + c - 1;
            const bool in = i < 18 * 18 && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
            dv[j] = in ? *(const uint2*)((const char*)dout + ((size_t)(b * H + gh) * W + gw) * 16 * sizeof(T))
                       : make_uint2(0u, 0u);
        }
    };
    // ---- constants: the dgrad's B fragments (W[k][c], k = 8 lq + e, c = 16 n + l16) hi + lo
    uint4 whi[4], wlo[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        float h8[8], l8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = 8 * lq + e, co = k / 9, tap = k - 9 * co;
            const float v = k < 9 * Co ? w[((size_t)co * C + 16 * n + l16) * 9 + tap] : 0.f;
            h8[e] = rnd16<T>(v);
            l8[e] = v - h8[e];
        }
        whi[n] = pack16<T>(h8);
        wlo[n] = pack16<T>(l8);
    }
    float al[4], ial[4];
    bool rec[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int c = 16 * n + l16;
        al[n] = alpha[c];
        ial[n] = __builtin_amdgcn_rcpf(al[n]);
        rec[n] = all_pos4(alpha + (c & ~3));
    }
    float dal[4] = {0.f, 0.f, 0.f, 0.f};
    f32x4 acw[2][4];                       // dW[k = 16 km + 4 lq + i][c = 16 n + l16], this wave's rows r
#pragma unroll
    for (int km = 0; km < 2; ++km)
#pragma unroll
        for (int n = 0; n < 4; ++n) acw[km][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum[3] = {0.f, 0.f, 0.f};
    // ---- the im2col builder's role: pixel pair (2 p2, 2 p2 + 1) in r order
    const int p2 = tid & 127;
    const int Hh = H >> 1, Wh = W >> 1;
    int t = blockIdx.x;
    if (t < ntiles) load(t);
    for (; t < ntiles; t += gridDim.x) {
        __syncthreads();                                   // (A) the previous tile's LDS reads done
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (tid + 256 * j < 18 * 18) hd[tid + 256 * j] = dv[j];
        {
            // P^T[c][r]: the pair (2P, 2P + 1) is (r, r + 1), r = 4 dp + 2 ((P >> 3) & 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int P = pp + 32 * j;
                const int r = 4 * ((P >> 4) * 8 + (P & 7)) + 2 * ((P >> 3) & 1);
                const unsigned a0[4] = {pv[j][0].x, pv[j][0].y, pv[j][0].z, pv[j][0].w};
                const unsigned a1[4] = {pv[j][1].x, pv[j][1].y, pv[j][1].z, pv[j][1].w};
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const unsigned wd = __builtin_amdgcn_perm(a1[i >> 1], a0[i >> 1], (i & 1) ? 0x07060302u : 0x05040100u);
                    *(unsigned*)pt(8 * pcq + i, r) = wd;
                }
            }
        }
        __syncthreads();                                   // (B) halo and P^T written
        if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);   // the next tile, under this one's work
        // X rows r0, r0 + 1 (k half KH, wave-uniform: waves 0-1 k 0..15, waves 2-3 k 16..31) and
        // the matching X^T words; bias partials.  KH a template constant: every k, co and tap
        // below is compile-time, the 9 halo words stay in registers (a runtime index into them
        // went to scratch, whose loads wait on the whole vmcnt queue: the prefetch)
        auto build = [&](auto KHC) {
            constexpr int KH = decltype(KHC)::value;
            const int r0 = 2 * p2;
            unsigned short xv[2][16];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = r0 + e, dp = r >> 2, q = r & 3;
                const int sh = 2 * (dp >> 3) + (q >> 1), sw = 2 * (dp & 7) + (q & 1);
                uint2 g[9];
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) g[tap] = hd[(sh - tap / 3 + 2) * 18 + (sw - tap % 3 + 2)];
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {
                    const int k = 16 * KH + kk, co = k / 9, tap = k - 9 * co;
                    unsigned short v = 0;
                    if (co < 3) {
                        const unsigned wd = co < 2 ? g[tap].x : g[tap].y;
                        v = co < Co ? (unsigned short)((co == 1) ? (wd >> 16) : (wd & 0xffffu)) : (unsigned short)0;
                    }
                    xv[e][kk] = v;
                }
                // bias: the centre tap (k = 9 co + 4) of the pixel's own dout
#pragma unroll
                for (int co = 0; co < 3; ++co)
                    if ((9 * co + 4) / 16 == KH) bsum[co] += tof<T>(__builtin_bit_cast(T, xv[e][(9 * co + 4) % 16]));
                uint4 u0, u1;
                u0.x = xv[e][0] | ((unsigned)xv[e][1] << 16);   u0.y = xv[e][2] | ((unsigned)xv[e][3] << 16);
                u0.z = xv[e][4] | ((unsigned)xv[e][5] << 16);   u0.w = xv[e][6] | ((unsigned)xv[e][7] << 16);
                u1.x = xv[e][8] | ((unsigned)xv[e][9] << 16);   u1.y = xv[e][10] | ((unsigned)xv[e][11] << 16);
                u1.z = xv[e][12] | ((unsigned)xv[e][13] << 16); u1.w = xv[e][14] | ((unsigned)xv[e][15] << 16);
                *(uint4*)(X + r * XS + 16 * KH) = u0;
                *(uint4*)(X + r * XS + 16 * KH + 8) = u1;
            }
#pragma unroll
            for (int kk = 0; kk < 16; ++kk)
                *(unsigned*)(XT + (16 * KH + kk) * TS + r0) = xv[0][kk] | ((unsigned)xv[1][kk] << 16);
        };
        if (wave < 2) build(std::integral_constant<int, 0>{});
        else build(std::integral_constant<int, 1>{});
        __syncthreads();                                   // (C) X, X^T written
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        // weight gradient: this wave's 64 rows r, 2 K steps of 32
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int rb = 64 * wave + 32 * ks + 8 * lq;
            uint4 A[2];
#pragma unroll
            for (int km = 0; km < 2; ++km) A[km] = *(const uint4*)(XT + (16 * km + l16) * TS + rb);
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                uint4 Bv = *(const uint4*)pt(16 * n + l16, rb);
                if (!rec[n]) {                             // P holds v: a = PReLU(v) in 16 bits
                    float f[8];
                    unpack16<T>(Bv, f);
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] = prelu_f(f[e], al[n]);
                    Bv = pack16<T>(f);
                }
#pragma unroll
                for (int km = 0; km < 2; ++km) mma16<T>(acw[km][n], A[km], Bv);
            }
        }
        // data gradient + PReLU' + unshuffle: 4 row blocks of 16 (4 du pixels each)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const uint4 A = *(const uint4*)(X + (64 * wave + 16 * mb + l16) * XS + 8 * lq);
            const int dp = 16 * wave + 4 * mb + lq;        // du pixel of the tile
            T* o = du + (((size_t)(b * Hh + (h0 >> 1) + (dp >> 3)) * Wh + (w0 >> 1) + (dp & 7)) * (4 * C));
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                mma16<T>(acc, A, whi[n]);
                mma16<T>(acc, A, wlo[n]);
                const int c = 16 * n + l16;
                const uint2 pw = *(const uint2*)pt(c, 4 * dp);
                const float pq[4] = {lo16<T>(pw.x), hi16<T>(pw.x), lo16<T>(pw.y), hi16<T>(pw.y)};
                float ov[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    dal[n] += prelu_dalpha_f(acc[j], pq[j]);
                    ov[j] = prelu_bwd_f(acc[j], pq[j], al[n]);
                }
                st4<T>(o + 4 * c, ov);
            }
        }
    }
    // ---- block partials: slopes (lanes of one l16 and the 4 waves), dW (the 4 waves), bias
    __syncthreads();
    float* red = (float*)(smem + 18 * 18 * 8);             // X / X^T / P^T are dead now
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        float v = rec[n] ? dal[n] * ial[n] : dal[n];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lq == 0) red[wave * 64 + 16 * n + l16] = v;
    }
    float* rw = red + 256;                                 // [4 waves][32 k][64 c]
#pragma unroll
    for (int km = 0; km < 2; ++km)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) rw[(wave * 32 + 16 * km + 4 * lq + i) * 64 + 16 * n + l16] = acw[km][n][i];
    float* rb3 = rw + 4 * 32 * 64;                         // [256 threads][3]
#pragma unroll
    for (int co = 0; co < 3; ++co) rb3[tid * 3 + co] = bsum[co];
    __syncthreads();
    if (tid < C) dal_part[(size_t)blockIdx.x * C + tid] = ((red[tid] + red[64 + tid]) + red[128 + tid]) + red[192 + tid];
    const int nk = 9 * Co;
    for (int i = tid; i < nk * C; i += 256) {
        const int k = i / C, c = i - k * C, co = k / 9, tap = k - 9 * co;
        const float v = ((rw[k * 64 + c] + rw[(32 + k) * 64 + c]) + rw[(64 + k) * 64 + c]) + rw[(96 + k) * 64 + c];
        dw_part[(size_t)blockIdx.x * (Co * C * 9) + ((size_t)co * C + c) * 9 + tap] = v;
    }
    if (tid < Co) {
        float v = 0.f;
        for (int i = 0; i < 256; ++i) v += rb3[i * 3 + tid];
        db_part[(size_t)blockIdx.x * Co + tid] = v;
    }
}

// ------------------------------- channel attention -------------------------------
// blocks.py:83-92: mean -> fc0 (C->Cr, no bias) -> ReLU -> fc2 (Cr->C) -> sigmoid, for image
// b, by one 256-thread block, into sg[C] (LDS).  Written for latency: every global load of a
// phase is independent (the pool partials are split 256/C ways per channel, the FC dot
// products 16 / 4 ways per output), so each phase costs one memory round trip.
// Needs C % 16 == 0, Cr % 4 == 0, C <= 256, Cr <= 64.
__device__ __forceinline__ void se_gate(int b, int C, int Cr, int nparts, float inv_hw, const float* __restrict__ part,
                                        const float* __restrict__ w1, const float* __restrict__ w2, float* sm,
                                        float* sh, float* sg, float* red, float* mean, float* hid, float* s_out) {
    const int tid = threadIdx.x;
    const int G = C >= 256 ? 1 : 256 / C;   // threads per channel for the pool reduction
    if (tid < G * C) {
        const int c = tid % C, g = tid / C;
        const float* pp = part + (size_t)b * nparts * C + c;
        float a = 0.f;
#pragma unroll 4
        for (int p = g; p < nparts; p += G) a += pp[(size_t)p * C];
        red[g * C + c] = a;
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        float a = 0.f;
        for (int g = 0; g < G; ++g) a += red[g * C + c];
        a *= inv_hw;
        sm[c] = a;
        if (mean) mean[(size_t)b * C + c] = a;
    }
    __syncthreads();
    const int k1 = C / 16;                  // fc0: 16 lanes per hidden unit
    for (int idx = tid; idx < Cr * 16; idx += 256) {
        const int j = idx >> 4, seg = idx & 15;
        const float* wr = w1 + (size_t)j * C + seg * k1;
        float a = 0.f;
        for (int k = 0; k < k1; ++k) a += wr[k] * sm[seg * k1 + k];
        a = group16_sum(a);
        if (seg == 0) {
            a = fmaxf(a, 0.f);
            sh[j] = a;
            if (hid) hid[(size_t)b * Cr + j] = a;
        }
    }
    __syncthreads();
    const int k2 = Cr / 4;                  // fc2: 4 lanes per channel
    for (int idx = tid; idx < C * 4; idx += 256) {
        const int c = idx >> 2, seg = idx & 3;
        const float* wr = w2 + (size_t)c * Cr + seg * k2;
        float a = 0.f;
        for (int k = 0; k < k2; ++k) a += wr[k] * sh[seg * k2 + k];
        a += __shfl_xor(a, 1, 64);
        a += __shfl_xor(a, 2, 64);
        if (seg == 0) {
            const float v = 1.f / (1.f + expf(-a));
            sg[c] = v;
            if (s_out) s_out[(size_t)b * C + c] = v;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_se_fwd(int C, int Cr, int nparts, float inv_hw, const float* __restrict__ part,
                                                const float* __restrict__ w1, const float* __restrict__ w2,
                                                float* mean, float* hid, float* s) {
    __shared__ float sm[256], sh[64], sg[256], red[256];
    se_gate(blockIdx.x, C, Cr, nparts, inv_hw, part, w1, w2, sm, sh, sg, red, mean, hid, s);
}

// SE gate + apply in one launch: grid (splits, B); every block recomputes its image's gate
// and block 0 of each image stores mean/hid/s.  Latency layout: the gate's operands (pool
// partials, both FC weights) are loaded first -- head of the memory queue -- then each
// thread's NPT t / x vectors, so the streaming loads are in flight while the gate is
// computed from LDS; then y = t * s[c] * rs + x.  Needs C * Cr <= 4096 and nparts <= 8*(256/C)
// for the single-round-trip path (larger nparts take a slower tail loop).
template <typename T, int NPT>
__global__ __launch_bounds__(256) void k_se_fused(int HW, int C, int Cr, int nparts, float inv_hw,
                                                  const float* __restrict__ part, const float* __restrict__ w1,
                                                  const float* __restrict__ w2, float* mean, float* hid, float* s,
                                                  const T* __restrict__ t, float rs, const T* __restrict__ x,
                                                  T* __restrict__ y) {
    __shared__ float sm[256], sh[64], sg[256], red[256];
    __shared__ __attribute__((aligned(16))) float w1s[4096], w2s[4096];
    constexpr int V = 16 / sizeof(T);
    const int tid = threadIdx.x, b = blockIdx.y;
    // ---- 1. gate operands
    const int G = C >= 256 ? 1 : 256 / C;
    const int c = tid % C, g = tid / C;
    const bool act = tid < G * C;
    const float* pp = part + (size_t)b * nparts * C + c;
    float pv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int p = g + i * G;
        pv[i] = (act && p < nparts) ? pp[(size_t)p * C] : 0.f;
    }
    const int nw4 = C * Cr / 4;
    float4 w1v[4], w2v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + j * 256;
        if (i < nw4) {
            w1v[j] = ((const float4*)w1)[i];
            w2v[j] = ((const float4*)w2)[i];
        }
    }
    // ---- 2. streaming operands
    const size_t nv = (size_t)HW * C / V;
    const size_t base = (size_t)b * nv;
    const size_t v0 = (size_t)blockIdx.x * (256 * NPT) + tid;
    uint4 tv[NPT], xv[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const size_t v = v0 + (size_t)j * 256;
        if (v < nv) {
            tv[j] = *(const uint4*)(t + (base + v) * V);
            xv[j] = *(const uint4*)(x + (base + v) * V);
        }
    }
    // ---- 3. gate
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += pv[i];
    for (int p = g + 8 * G; act && p < nparts; p += G) a += pp[(size_t)p * C];
    if (act) red[g * C + c] = a;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + j * 256;
        if (i < nw4) {
            ((float4*)w1s)[i] = w1v[j];
            ((float4*)w2s)[i] = w2v[j];
        }
    }
    __syncthreads();
    const bool first = blockIdx.x == 0;
    for (int cc = tid; cc < C; cc += 256) {
        float m = 0.f;
        for (int k = 0; k < G; ++k) m += red[k * C + cc];
        m *= inv_hw;
        sm[cc] = m;
        if (first && mean) mean[(size_t)b * C + cc] = m;
    }
    __syncthreads();
    const int k1 = C / 16;
    for (int idx = tid; idx < Cr * 16; idx += 256) {
        const int j = idx >> 4, seg = idx & 15;
        const float* wr = w1s + j * C + seg * k1;
        float h = 0.f;
        for (int k = 0; k < k1; ++k) h += wr[k] * sm[seg * k1 + k];
        h = group16_sum(h);
        if (seg == 0) {
            h = fmaxf(h, 0.f);
            sh[j] = h;
            if (first && hid) hid[(size_t)b * Cr + j] = h;
        }
    }
    __syncthreads();
    const int k2 = Cr / 4;
    for (int idx = tid; idx < C * 4; idx += 256) {
        const int cc = idx >> 2, seg = idx & 3;
        const float* wr = w2s + cc * Cr + seg * k2;
        float z = 0.f;
        for (int k = 0; k < k2; ++k) z += wr[k] * sh[seg * k2 + k];
        z += __shfl_xor(z, 1, 64);
        z += __shfl_xor(z, 2, 64);
        if (seg == 0) {
            const float v = 1.f / (1.f + expf(-z));
            sg[cc] = v;
            if (first && s) s[(size_t)b * C + cc] = v;
        }
    }
    __syncthreads();
    // ---- 4. apply
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const size_t v = v0 + (size_t)j * 256;
        if (v < nv) {
            const int c0 = (int)((v * V) % C);
            float av[V], bv[V], o[V];
            unpack16<T>(tv[j], av);
            unpack16<T>(xv[j], bv);
#pragma unroll
            for (int k = 0; k < V; ++k) o[k] = av[k] * sg[c0 + k] * rs + bv[k];
            *(uint4*)(y + (base + v) * V) = pack16<T>(o);
        }
    }
}

// y = t * s[b,c] * rs + x   or (bwd)  dt = dy * s[b,c] * rs + g[b,c]
template <typename T, bool BWD>
__global__ void k_se_apply(size_t nvec, int HW, int C, const T* __restrict__ t, const float* __restrict__ s,
                           float rs, const void* __restrict__ x, T* __restrict__ y) {
    constexpr int V = 16 / sizeof(T);
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const size_t e0 = i * V;
    const int c0 = (int)(e0 % C);
    const size_t b = e0 / ((size_t)HW * C);
    float tv[V], o[V];
    unpack16<T>(*(const uint4*)(t + e0), tv);
    const float* sp = s + b * C + c0;
    if constexpr (!BWD) {
        float xv[V];
        unpack16<T>(*(const uint4*)((const T*)x + e0), xv);
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = tv[j] * sp[j] * rs + xv[j];
    } else {
        const float* gp = (const float*)x + b * C + c0;
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = tv[j] * rs * sp[j] + gp[j];
    }
    *(uint4*)(y + e0) = pack16<T>(o);
}

// part[b][chunk][c] = sum over the chunk's pixels of a*b_ (or a)
template <typename T>
__global__ __launch_bounds__(256) void k_pool_dot(int HW, int C, int nchunk, const T* __restrict__ a,
                                                  const T* __restrict__ bb, float* __restrict__ part) {
    constexpr int V = 16 / sizeof(T);
    __shared__ float red[256][V];
    const int TP = C / V;                    // threads per pixel
    const int R = 256 / TP;                  // pixels per iteration
    const int tid = threadIdx.x, cv = tid % TP, pr = tid / TP;
    const int b = blockIdx.y, ch = blockIdx.x;
    const int per = (HW + nchunk - 1) / nchunk;
    const int p0 = ch * per, p1 = min(p0 + per, HW);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    if (pr < R) {
#pragma unroll 4
        for (int p = p0 + pr; p < p1; p += R) {     // unrolled: 4 pixel rows of loads in flight
            const size_t e = ((size_t)b * HW + p) * C + cv * V;
            float av[V];
            unpack16<T>(*(const uint4*)(a + e), av);
            if (bb) {
                float bv[V];
                unpack16<T>(*(const uint4*)(bb + e), bv);
#pragma unroll
                for (int j = 0; j < V; ++j) acc[j] += av[j] * bv[j];
            } else {
#pragma unroll
                for (int j = 0; j < V; ++j) acc[j] += av[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) red[tid][j] = acc[j];
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        const int cvv = c / V, j = c % V;
        float sum = 0.f;
        for (int r = 0; r < R; ++r) sum += red[r * TP + cvv][j];
        part[((size_t)b * nchunk + ch) * C + c] = sum;
    }
}

constexpr int SE_STAGE_MAX = 4096;   // FC weights staged in LDS up to C * Cr floats each

// SE backward for one image (block per b).  Every operand the chain needs (s, hid, mean and,
// when they fit, both FC weights) is requested up front beside the pool partials and staged in
// LDS, so the dependent steps (sigmoid', FC2^T + ReLU', the weight-gradient rows, FC1^T) run
// on LDS instead of paying one global round trip each.
template <bool STAGE>
__global__ void k_se_bwd(int C, int Cr, int nparts, float inv_hw, float rs, const float* __restrict__ part,
                         const float* __restrict__ mean, const float* __restrict__ hid, const float* __restrict__ s,
                         const float* __restrict__ w1, const float* __restrict__ w2, float* g, float* dw1p,
                         float* dw2p) {
    __shared__ float dz[512], dh[128], pr[4][256], ssv[512], smean[512], shid[128];
    __shared__ float sw1[STAGE ? SE_STAGE_MAX : 1], sw2[STAGE ? SE_STAGE_MAX : 1];
    const int b = blockIdx.x, t = threadIdx.x;
    for (int c = t; c < C; c += blockDim.x) {
        ssv[c] = s[(size_t)b * C + c];
        smean[c] = mean[(size_t)b * C + c];
    }
    for (int j = t; j < Cr; j += blockDim.x) shid[j] = hid[(size_t)b * Cr + j];
    if constexpr (STAGE) {
        for (int i = t; i < C * Cr; i += blockDim.x) {
            sw1[i] = w1[i];
            sw2[i] = w2[i];
        }
    }
    // pool partials: thread (c, quarter) sums every 4th part (independent loads in flight),
    // fixed-order combine of the quarters (deterministic)
    for (int c0 = 0; c0 < C; c0 += 64) {
        const int c = c0 + (t & 63), qr = t >> 6;
        float a = 0.f;
        if (c < C) {
#pragma unroll 4
            for (int p = qr; p < nparts; p += 4) a += part[((size_t)b * nparts + p) * C + c];
        }
        pr[qr][c & 255] = a;
    }
    __syncthreads();
    for (int c = t; c < C; c += blockDim.x) {
        const float a = (pr[0][c] + pr[1][c]) + (pr[2][c] + pr[3][c]);
        const float sv = ssv[c];
        dz[c] = a * rs * sv * (1.f - sv);                 // through sigmoid
    }
    __syncthreads();
    {   // dh[j] = relu'(hid) * sum_c w2[c][j] dz[c]: one wave per hidden unit, lanes over c
        const int lane = t & 63, nw = blockDim.x >> 6;
        for (int j = t >> 6; j < Cr; j += nw) {
            float a = 0.f;
            for (int c = lane; c < C; c += 64) a += (STAGE ? sw2[c * Cr + j] : w2[(size_t)c * Cr + j]) * dz[c];
            a = wave_sum(a);
            if (lane == 0) dh[j] = shid[j] > 0.f ? a : 0.f;   // through ReLU
        }
    }
    __syncthreads();
    for (int i = t; i < C * Cr; i += blockDim.x) {
        const int c = i / Cr, j = i % Cr;
        dw2p[(size_t)b * C * Cr + i] = dz[c] * shid[j];                        // [C][Cr]
        const int jj = i / C, cc = i % C;
        dw1p[(size_t)b * C * Cr + i] = dh[jj] * smean[cc];                      // [Cr][C]
    }
    for (int c = t; c < C; c += blockDim.x) {
        float a = 0.f;
        for (int j = 0; j < Cr; ++j) a += (STAGE ? sw1[j * C + c] : w1[(size_t)j * C + c]) * dh[j];
        g[(size_t)b * C + c] = a * inv_hw;
    }
}

// SE backward + its apply in one launch (the backward of ChannelAttention and of the RCAB's
// scaled residual, blocks.py:88-92,150-153): grid (splits, B), every block recomputes its
// image's SE backward from the pool_dot partials -- the same arithmetic in the same order as
// k_se_bwd (thread (c, quarter) sums every 4th partial, fixed-order combine, one wave per
// hidden unit) -- and applies dt = dy * rs * s[c] + g[c] to its slice; block 0 of each image
// writes the FC weight-gradient rows (and g when asked).  The partials, both FC weights and
// the per-image vectors are requested first, then each thread's NPT dy vectors, so the
// streaming loads are in flight while the chain runs on LDS.  C <= 64, nparts <= 64,
// C * Cr <= 4096.
template <typename T, int NPT>
__global__ __launch_bounds__(256) void k_se_bwd_fused(int HW, int C, int Cr, int nparts, float inv_hw, float rs,
                                                      const float* __restrict__ part, const float* __restrict__ mean,
                                                      const float* __restrict__ hid, const float* __restrict__ s,
                                                      const float* __restrict__ w1, const float* __restrict__ w2,
                                                      const T* __restrict__ dy, float* g_out, float* dw1p, float* dw2p,
                                                      T* __restrict__ dt) {
    __shared__ float dz[64], dh[64], pr[4][64], ssv[64], smean[64], shid[64], sgv[64];
    __shared__ __attribute__((aligned(16))) float sw1[4096], sw2[4096];
    constexpr int V = 16 / sizeof(T);
    const int t = threadIdx.x, b = blockIdx.y;
    const int c = t & 63, qr = t >> 6;
    // ---- 1. the chain's operands
    float pv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int pidx = qr + 4 * i;
        pv[i] = (c < C && pidx < nparts) ? part[((size_t)b * nparts + pidx) * C + c] : 0.f;
    }
    const int nw4 = C * Cr / 4;
    float4 w1v[4], w2v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = t + j * 256;
        if (i < nw4) {
            w1v[j] = ((const float4*)w1)[i];
            w2v[j] = ((const float4*)w2)[i];
        }
    }
    float sv0 = 0.f, mv0 = 0.f, hv0 = 0.f;
    if (t < C) {
        sv0 = s[(size_t)b * C + t];
        mv0 = mean[(size_t)b * C + t];
    }
    if (t < Cr) hv0 = hid[(size_t)b * Cr + t];
    // ---- 2. streaming operands
    const size_t nv = (size_t)HW * C / V;
    const size_t base = (size_t)b * nv;
    const size_t v0 = (size_t)blockIdx.x * (256 * NPT) + t;
    uint4 yv[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const size_t v = v0 + (size_t)j * 256;
        if (v < nv) yv[j] = *(const uint4*)(dy + (base + v) * V);
    }
    // ---- 3. SE backward (k_se_bwd's order)
    {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) a += pv[i];
        if (c < C) pr[qr][c] = a;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = t + j * 256;
        if (i < nw4) {
            ((float4*)sw1)[i] = w1v[j];
            ((float4*)sw2)[i] = w2v[j];
        }
    }
    if (t < C) {
        ssv[t] = sv0;
        smean[t] = mv0;
    }
    if (t < Cr) shid[t] = hv0;
    __syncthreads();
    if (t < C) {
        const float a = (pr[0][t] + pr[1][t]) + (pr[2][t] + pr[3][t]);
        const float sv = ssv[t];
        dz[t] = a * rs * sv * (1.f - sv);                 // through sigmoid
    }
    __syncthreads();
    {
        const int lane = t & 63;
        for (int j = t >> 6; j < Cr; j += 4) {
            float a = 0.f;
            for (int cc = lane; cc < C; cc += 64) a += sw2[cc * Cr + j] * dz[cc];
            a = wave_sum(a);
            if (lane == 0) dh[j] = shid[j] > 0.f ? a : 0.f;   // through ReLU
        }
    }
    __syncthreads();
    const bool first = blockIdx.x == 0;
    if (first) {
        for (int i = t; i < C * Cr; i += 256) {
            const int cc = i / Cr, j = i % Cr;
            dw2p[(size_t)b * C * Cr + i] = dz[cc] * shid[j];                       // [C][Cr]
            const int jj = i / C, c2 = i % C;
            dw1p[(size_t)b * C * Cr + i] = dh[jj] * smean[c2];                     // [Cr][C]
        }
    }
    if (t < C) {
        float a = 0.f;
        for (int j = 0; j < Cr; ++j) a += sw1[j * C + t] * dh[j];
        const float gv = a * inv_hw;
        sgv[t] = gv;
        if (first && g_out) g_out[(size_t)b * C + t] = gv;
    }
    __syncthreads();
    // ---- 4. dt = dy * rs * s[c] + g[c]  (k_se_apply<BWD>'s expression)
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const size_t v = v0 + (size_t)j * 256;
        if (v < nv) {
            const int c0 = (int)((v * V) % C);
            float av[V], o[V];
            unpack16<T>(yv[j], av);
#pragma unroll
            for (int k = 0; k < V; ++k) o[k] = av[k] * rs * ssv[c0 + k] + sgv[c0 + k];
            *(uint4*)(dt + (base + v) * V) = pack16<T>(o);
        }
    }
}

// ------------------------------ resampling / layout ------------------------------
__global__ void k_bicubic_down4(int B, int C, int H, int W, const float* __restrict__ hr, float* __restrict__ lr) {
    const int Ho = H / 4, Wo = W / 4;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * C * Ho * Wo) return;
    const int ox = (int)(i % Wo), oy = (int)((i / Wo) % Ho);
    const size_t plane = i / ((size_t)Wo * Ho);
    lr[i] = bicubic_sample(hr + plane * H * W, H, W, oy, ox, 4.0f);
}

template <typename T>
__global__ void k_nchw_to_nhwc(int B, int C, int H, int W, int Cpad, const float* __restrict__ x, T* __restrict__ y) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // NHWC order
    if (i >= (size_t)B * Cpad * H * W) return;
    const int c = (int)(i % Cpad);
    const size_t px = i / Cpad;
    const int w = (int)(px % W), h = (int)((px / W) % H), b = (int)(px / ((size_t)W * H));
    y[i] = fromf<T>(c < C ? x[(((size_t)b * C + c) * H + h) * W + w] : 0.f);
}

// dv = dy * (pre>0 ? 1 : alpha[c]) -> du[b][h/2][w/2][4c + 2(h&1) + (w&1)]; block = 16x16 px tile
template <typename T>
__global__ __launch_bounds__(256) void k_prelu_bwd_unshuffle(int B, int H, int W, int C, const T* __restrict__ dy,
                                                             const T* __restrict__ pre, const float* __restrict__ alpha,
                                                             T* __restrict__ du, float* __restrict__ part) {
    __shared__ float sdal[256 * 2];
    const int tid = threadIdx.x;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int b = blockIdx.x / tpi, tile = blockIdx.x - b * tpi;
    const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
    const int K2 = C / 2, k = tid % K2;
    const float al0 = alpha[2 * k], al1 = alpha[2 * k + 1];
    float dal0 = 0.f, dal1 = 0.f;
    const int Hh = H >> 1, Wh = W >> 1;
    for (int i = tid; i < 64 * K2; i += 256) {
        const int dp = i / K2, hh = dp >> 3, ww = dp & 7;
        const int gh2 = (h0 >> 1) + hh, gw2 = (w0 >> 1) + ww;
        if (gh2 >= Hh || gw2 >= Wh) continue;
        float out[8];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const size_t pi = ((size_t)(b * H + 2 * gh2 + (t >> 1)) * W + 2 * gw2 + (t & 1)) * C + 2 * k;
            const float d0 = tof<T>(dy[pi]), d1 = tof<T>(dy[pi + 1]);
            const float p0 = tof<T>(pre[pi]), p1 = tof<T>(pre[pi + 1]);
            dal0 += prelu_dalpha_f(d0, p0);
            dal1 += prelu_dalpha_f(d1, p1);
            out[t] = prelu_bwd_f(d0, p0, al0);
            out[4 + t] = prelu_bwd_f(d1, p1, al1);
        }
        char* o = (char*)du + (((size_t)(b * Hh + gh2) * Wh + gw2) * (4 * C) + 8 * k) * sizeof(T);
        if constexpr (sizeof(T) == 2) {
            *(uint4*)o = pack16<T>(out);
        } else {
            *(uint4*)o = pack16<float>(out);
            *(uint4*)(o + 16) = pack16<float>(out + 4);
        }
    }
    sdal[tid * 2] = dal0;
    sdal[tid * 2 + 1] = dal1;
    __syncthreads();
    if (tid < C) {
        const int kk = tid >> 1, e = tid & 1;
        float s = 0.f;
        for (int r = kk; r < 256; r += K2) s += sdal[r * 2 + e];
        part[(size_t)blockIdx.x * C + tid] = s;
    }
}
template <typename T>
__global__ void k_nhwc_to_nchw(int B, int C, int H, int W, const T* __restrict__ x, float* __restrict__ y) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // NCHW order
    if (i >= (size_t)B * C * H * W) return;
    const int w = (int)(i % W), h = (int)((i / W) % H), c = (int)((i / ((size_t)W * H)) % C);
    const size_t b = i / ((size_t)W * H * C);
    y[i] = tof<T>(x[((b * H + h) * W + w) * C + c]);
}

template <typename T>
__global__ void k_pack(int mode, int Cout, int Cin, const float* __restrict__ w, T* __restrict__ out, size_t n);

// Column sums out[c] (+)= scale * sum_r part[r][c], several independent jobs per launch
// (the per-block PReLU dalpha / SE weight-gradient partials of a whole residual group).
// Block = 1024 threads = 16 row-waves x 64 columns, 4 independent accumulators per lane,
// fixed-order combine in LDS (bitwise reproducible).  cols == 1 (the loss) sums rows across
// all 1024 threads instead.
struct ColJobK {
    const float* part;
    float* out;
    int rows, cols;
    float scale;
    int accumulate;
    int blk0;   // first block of this job
    int nsplit; // row slices (tall narrow jobs): blocks per 64-column block
    int slot0;  // its first slot in the split scratch
};
constexpr int COLSUM_MAXJ = 40;
// Tall narrow jobs (the strip backward's slope rows, 2048 x 64 per RCAB) are split into up to 8
// row slices, one block each; the slices' partial rows go through this scratch and the last
// block of a column block sums them in slice order (deterministic).  One colsum launch at a
// time uses it (they run on the launching stream, in program order).
constexpr int COLSUM_SLOTS = 2 * COLSUM_MAXJ;
__device__ float g_cs_part[COLSUM_SLOTS][8][64];
__device__ unsigned g_cs_cnt[COLSUM_SLOTS];
struct ColJobs {
    int n;
    ColJobK j[COLSUM_MAXJ];
};

__global__ __launch_bounds__(1024) void k_colsum_multi(const ColJobs jobs) {
    __shared__ float red[16][64];
    int ji = 0;
    while (ji + 1 < jobs.n && (int)blockIdx.x >= jobs.j[ji + 1].blk0) ++ji;
    const ColJobK& jb = jobs.j[ji];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rows = jb.rows, cols = jb.cols;
    if (cols == 1) {
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int r = tid;
        for (; r + 3 * 1024 < rows; r += 4 * 1024) {
            a0 += jb.part[r]; a1 += jb.part[r + 1024]; a2 += jb.part[r + 2048]; a3 += jb.part[r + 3072];
        }
        for (; r < rows; r += 1024) a0 += jb.part[r];
        const float v = wave_sum((a0 + a1) + (a2 + a3));
        if (lane == 0) red[0][w] = v;
        __syncthreads();
        if (tid == 0) {
            float t = 0.f;
            for (int k = 0; k < 16; ++k) t += red[0][k];
            t *= jb.scale;
            jb.out[0] = jb.accumulate ? jb.out[0] + t : t;
        }
        return;
    }
    const int local = (int)blockIdx.x - jb.blk0, ns = jb.nsplit;
    const int cb = local / ns, sp = local - cb * ns;
    const int c = cb * 64 + lane;
    // this block's rows: [r_lo, r_hi) of slice sp
    const int r_lo = (int)((long long)rows * sp / ns), r_hi = (int)((long long)rows * (sp + 1) / ns);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (c < cols) {
        const float* p = jb.part + (size_t)r_lo * cols + c;
        const int rows_ = r_hi - r_lo;
        int r = w;
        // 32 rows in flight per lane (a tall narrow job's slice is one or two round trips)
        float a4 = 0.f, a5 = 0.f, a6 = 0.f, a7 = 0.f;
        for (; r + 496 < rows_; r += 512) {
            float v[32];
#pragma unroll
            for (int k = 0; k < 32; ++k) v[k] = p[(size_t)(r + 16 * k) * cols];
#pragma unroll
            for (int k = 0; k < 32; k += 8) {
                a0 += v[k]; a1 += v[k + 1]; a2 += v[k + 2]; a3 += v[k + 3];
                a4 += v[k + 4]; a5 += v[k + 5]; a6 += v[k + 6]; a7 += v[k + 7];
            }
        }
        for (; r + 112 < rows_; r += 128) {
            a0 += p[(size_t)r * cols];
            a1 += p[(size_t)(r + 16) * cols];
            a2 += p[(size_t)(r + 32) * cols];
            a3 += p[(size_t)(r + 48) * cols];
            a4 += p[(size_t)(r + 64) * cols];
            a5 += p[(size_t)(r + 80) * cols];
            a6 += p[(size_t)(r + 96) * cols];
            a7 += p[(size_t)(r + 112) * cols];
        }
        a0 += a4; a1 += a5; a2 += a6; a3 += a7;
        for (; r + 48 < rows_; r += 64) {
            a0 += p[(size_t)r * cols];
            a1 += p[(size_t)(r + 16) * cols];
            a2 += p[(size_t)(r + 32) * cols];
            a3 += p[(size_t)(r + 48) * cols];
        }
        for (; r < rows_; r += 16) a0 += p[(size_t)r * cols];
    }
    red[w][lane] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (ns == 1) {
        if (w == 0 && c < cols) {
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) t += red[k][lane];
            t *= jb.scale;
            jb.out[c] = jb.accumulate ? jb.out[c] + t : t;
        }
        return;
    }
    // split job: the slice's partial row out (agent-scope stores, drained), then one arrival;
    // the column block's last arrival sums the slices in order (agent-scope loads)
    __shared__ int last;
    const int slot = jb.slot0 + cb;
    if (w == 0) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) t += red[k][lane];
        __hip_atomic_store(&g_cs_part[slot][sp][lane], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
            last = __hip_atomic_fetch_add(&g_cs_cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(ns - 1);
    }
    __syncthreads();
    if (last && w == 0) {
        float t = 0.f;
        for (int k = 0; k < ns; ++k) t += __hip_atomic_load(&g_cs_part[slot][k][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t *= jb.scale;
        if (c < cols) jb.out[c] = jb.accumulate ? jb.out[c] + t : t;
        if (lane == 0) __hip_atomic_store(&g_cs_cnt[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Pack many conv weights in one launch: job k covers packed elements [e0[k], e0[k+1]).
// Each job's range in the launch's index space is rounded up to whole 256-thread blocks, so a
// block's job is block-uniform (one scalar search per block, not a dependent chain of e0
// loads per thread) and the element math is 32-bit.
constexpr unsigned PACK_RUN = 8;                  // consecutive packed elements per thread (one 16-B store)
constexpr unsigned PACK_BLK = 256 * PACK_RUN;
struct PackJobK {
    const float* w;
    void* out;
    int mode, Cout, Cin;
    unsigned n;   // packed elements
};
template <typename T>
__device__ __forceinline__ void pack_one(int mode, int Cout, int Cin, const float* __restrict__ w, T* __restrict__ out,
                                         unsigned i) {
    if (mode == 2) {  // [9][Cin_pad][Cout], row = ci, taps flipped
        const int co = (int)(i % (unsigned)Cout);
        const int ci = (int)((i / (unsigned)Cout) % (unsigned)((Cin + 15) & ~15));
        const int tap = (int)(i / ((unsigned)Cout * (unsigned)((Cin + 15) & ~15)));
        const int kh = 2 - tap / 3, kw = 2 - tap % 3;
        out[i] = fromf<T>(ci < Cin ? w[(((size_t)co * Cin + ci) * 3 + kh) * 3 + kw] : 0.f);
    } else {          // [9][Cout_pad][Cin], row = co (mode 1: shuffle-permuted rows)
        const int coutp = (Cout + 15) & ~15;
        const int ci = (int)(i % (unsigned)Cin);
        const int cp = (int)((i / (unsigned)Cin) % (unsigned)coutp);
        const int tap = (int)(i / ((unsigned)Cin * (unsigned)coutp));
        int co = cp;
        if (mode == 1) { const int Cq = Cout / 4; co = 4 * (cp % Cq) + cp / Cq; }
        out[i] = fromf<T>(cp < Cout ? w[(((size_t)co * Cin + ci) * 3 + tap / 3) * 3 + tap % 3] : 0.f);
    }
}
// PACK_RUN consecutive packed elements from i (a multiple of PACK_RUN): one index decomposition,
// then the row / channel / tap counters stepped with carries
template <typename T>
__device__ __forceinline__ void pack_run(int mode, int Cout, int Cin, const float* __restrict__ w, T* __restrict__ out,
                                         unsigned i) {
    float v[PACK_RUN];
    if (mode == 2) {
        const unsigned cinp = (unsigned)((Cin + 15) & ~15);
        unsigned co = i % (unsigned)Cout, ci = (i / (unsigned)Cout) % cinp, tap = i / ((unsigned)Cout * cinp);
#pragma unroll
        for (unsigned k = 0; k < PACK_RUN; ++k) {
            const unsigned kh = 2 - tap / 3, kw = 2 - tap % 3;
            v[k] = ci < (unsigned)Cin ? w[(((size_t)co * Cin + ci) * 3 + kh) * 3 + kw] : 0.f;
            if (++co == (unsigned)Cout) {
                co = 0;
                if (++ci == cinp) { ci = 0; ++tap; }
            }
        }
    } else {
        const unsigned coutp = (unsigned)((Cout + 15) & ~15), Cq = (unsigned)Cout / 4;
        unsigned ci = i % (unsigned)Cin, cp = (i / (unsigned)Cin) % coutp, tap = i / ((unsigned)Cin * coutp);
#pragma unroll
        for (unsigned k = 0; k < PACK_RUN; ++k) {
            const unsigned co = mode == 1 ? 4 * (cp % Cq) + cp / Cq : cp;
            v[k] = cp < (unsigned)Cout ? w[(((size_t)co * Cin + ci) * 3 + tap / 3) * 3 + tap % 3] : 0.f;
            if (++ci == (unsigned)Cin) {
                ci = 0;
                if (++cp == coutp) { cp = 0; ++tap; }
            }
        }
    }
    if constexpr (sizeof(T) == 2) {
        *(uint4*)(out + i) = pack16<T>(v);
    } else {
        *(uint4*)(out + i) = pack16<float>(v);
        *(uint4*)(out + i + 4) = pack16<float>(v + 4);
    }
}
template <typename T>
__global__ void k_pack(int mode, int Cout, int Cin, const float* __restrict__ w, T* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pack_one<T>(mode, Cout, Cin, w, out, (unsigned)i);
}
template <typename T>
__global__ void k_pack_multi(int njobs, const PackJobK* __restrict__ jobs, const unsigned long long* __restrict__ e0,
                             unsigned long long total) {
    const unsigned long long b0 = (unsigned long long)blockIdx.x * PACK_BLK;   // block-uniform
    if (b0 >= total) return;
    int lo = 0, hi = njobs - 1;   // last job with e0 <= b0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (e0[mid] <= b0) lo = mid; else hi = mid - 1;
    }
    const PackJobK jb = jobs[lo];
    // packed sizes are multiples of 16 (padded Cout / Cin rows): a run never straddles a job's end
    const unsigned j = (unsigned)(b0 - e0[lo]) + threadIdx.x * PACK_RUN;
    if (j < jb.n) pack_run<T>(jb.mode, jb.Cout, jb.Cin, jb.w, (T*)jb.out, j);
}

constexpr int SUMSQ_BLOCKS_MAX = 1024;
__global__ void k_sumsq(size_t n, const float* __restrict__ g, float* part) {
    __shared__ float red[4];
    float s = 0.f;
    const size_t n4 = n / 4;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = ((const float4*)g)[i];
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    if (blockIdx.x == 0)
        for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += g[i] * g[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void k_optim_prepare(int nparts, const float* part, float max_norm, float b1, float b2, float wd,
                                float* scal) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]);
        float coef = 1.f;
        if (max_norm > 0.f) coef = fminf(max_norm / (norm + 1e-6f), 1.f);
        const float step = scal[2] + 1.f;
        const float lr = scal[3];
        scal[0] = norm;
        scal[1] = coef;
        scal[2] = step;
        scal[4] = 1.f - lr * wd;
        scal[5] = lr / (1.f - powf(b1, step));
        scal[6] = 1.f / sqrtf(1.f - powf(b2, step));
    }
}
__global__ void k_adamw(size_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                        float* __restrict__ v, const float* __restrict__ scal, float b1, float b2, float eps) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float coef = scal[1], decay = scal[4], step_size = scal[5], rbc2 = scal[6];
    const float gi = g[i] * coef;
    float pi = p[i] * decay;
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);    // lerp
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) * rbc2 + eps;
    pi = pi - step_size * mi / denom;
    p[i] = pi; m[i] = mi; v[i] = vi;
}
// torch.optim.AdamW over a list of separate tensors (the discriminator's optimizer_d,
// trainer.py:230-250, 446-451): per tensor its own device step count (torch's capturable form),
// incremented by k_adamw_steps before the update reads it.  Blocks map to jobs by a prefix of
// block offsets; each thread updates 4 consecutive elements (a tensor's tail by element).
constexpr int ADAMW_MAXJ = 48;
struct AdamJobK {
    float* p;
    const float* g;
    float* m;
    float* v;
    float* step;
    long long n;
    int blk0;
    int vec;                                 // all four 16-B aligned
};
struct AdamJobs {
    int n;
    float lr, b1, b2, eps, wd, omb1, omb2;   // 1 - b1, 1 - b2 as the caller rounds them (torch: from the Python doubles)
    AdamJobK j[ADAMW_MAXJ];
};
__global__ void k_adamw_steps(const AdamJobs jobs) {
    const int i = threadIdx.x;
    if (i < jobs.n) jobs.j[i].step[0] += 1.f;
}
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float decay, float step_size, float rbc2,
                                           const AdamJobs& jobs) {
    m = m + jobs.omb1 * (g - m);                                   // lerp
    v = v * jobs.b2 + jobs.omb2 * g * g;
    p = p * decay - step_size * m / (sqrtf(v) * rbc2 + jobs.eps);
}
// a block = ADAM_U x 256 float4 chunks of one job (4096 elements), each thread ADAM_U of them
// with every load in flight before the first update (one chunk per thread ran at ~3 TB/s:
// the 38 M-element optimizer_d step 195 us); per-element arithmetic unchanged
constexpr int ADAM_U = 4;
constexpr int ADAM_BLK = 256 * 4 * ADAM_U;
__global__ __launch_bounds__(256) void k_adamw_multi(const AdamJobs jobs) {
    int ji = 0;
    while (ji + 1 < jobs.n && (int)blockIdx.x >= jobs.j[ji + 1].blk0) ++ji;
    const AdamJobK& jb = jobs.j[ji];
    const long long base = (long long)(blockIdx.x - jb.blk0) * ADAM_BLK;
    const float step = jb.step[0];
    const float lr = jobs.lr;
    const float decay = 1.f - lr * jobs.wd;
    const float step_size = lr / (1.f - powf(jobs.b1, step));
    const float rbc2 = 1.f / sqrtf(1.f - powf(jobs.b2, step));
    if (jb.vec && base + ADAM_BLK <= jb.n) {
        // 16-B accesses (every tensor of the job 16-B aligned: fen_adamw_multi checks)
        float4 p[ADAM_U], g[ADAM_U], m[ADAM_U], v[ADAM_U];
#pragma unroll
        for (int u = 0; u < ADAM_U; ++u) {
            const long long i = base + ((long long)u * 256 + threadIdx.x) * 4;
            p[u] = *(const float4*)(jb.p + i), g[u] = *(const float4*)(jb.g + i);
            m[u] = *(const float4*)(jb.m + i), v[u] = *(const float4*)(jb.v + i);
        }
#pragma unroll
        for (int u = 0; u < ADAM_U; ++u) {
            const long long i = base + ((long long)u * 256 + threadIdx.x) * 4;
            adamw_elem(p[u].x, g[u].x, m[u].x, v[u].x, decay, step_size, rbc2, jobs);
            adamw_elem(p[u].y, g[u].y, m[u].y, v[u].y, decay, step_size, rbc2, jobs);
            adamw_elem(p[u].z, g[u].z, m[u].z, v[u].z, decay, step_size, rbc2, jobs);
            adamw_elem(p[u].w, g[u].w, m[u].w, v[u].w, decay, step_size, rbc2, jobs);
            *(float4*)(jb.p + i) = p[u];
            *(float4*)(jb.m + i) = m[u];
            *(float4*)(jb.v + i) = v[u];
        }
        return;
    }
    // the job's last (partial) block, or unaligned tensors: element by element
    for (int u = 0; u < ADAM_U; ++u) {
        const long long i0 = base + ((long long)u * 256 + threadIdx.x) * 4;
        for (int e = 0; e < 4; ++e) {
            const long long i = i0 + e;
            if (i >= jb.n) break;
            float p = jb.p[i], m = jb.m[i], v = jb.v[i];
            adamw_elem(p, jb.g[i], m, v, decay, step_size, rbc2, jobs);
            jb.p[i] = p, jb.m[i] = m, jb.v[i] = v;
        }
    }
}
__global__ void k_scale(size_t n, float* y, float s) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] *= s;
}

}  // namespace

// =================================== C-ABI ===================================
#define STREAM ((hipStream_t)stream)

extern "C" int fen_conv_first_fwd_ex(int dtype, int B, int Ci, int H, int W, int C, const float* x, const float* w,
                                     const float* bias, const float* in_mean, const float* in_istd, float act, void* y,
                                     void* stream) {
    if (!x || !w || !bias || !y || B <= 0 || Ci <= 0 || Ci > 3 || C % 8 || C > 128) return FEN_EINVAL;
    const size_t n = (size_t)B * H * W * (C / 8);
    const size_t lds = (size_t)Ci * 9 * C * sizeof(float);
    static int m16 = -1;                                 // FEN_CF_M16=0: the VALU forms (A/B runs)
    if (m16 < 0) {
        const char* e = getenv("FEN_CF_M16");
        m16 = e ? atoi(e) : 1;
    }
    if (m16 && (dtype == FEN_BF16 || dtype == FEN_F16) && (C == 16 || C == 32 || C == 64 || C == 128)) {
        const int ntiles = B * ((H + 15) >> 4) * ((W + 15) >> 4);
        const unsigned nb = (unsigned)std::min(ntiles, CFM16_BLOCKS);
#define CFM16_LAUNCH(TT, MBv)                                                                                   \
    hipLaunchKernelGGL((k_conv_first_m16<TT, MBv>), dim3(nb), dim3(256), 0, STREAM, B, Ci, H, W, C, x, w, bias, \
                       (TT*)y, in_mean, in_istd, act)
#define CFM16_MB(TT)                      \
    switch (C / 16) {                     \
        case 1: CFM16_LAUNCH(TT, 1); break; \
        case 2: CFM16_LAUNCH(TT, 2); break; \
        case 4: CFM16_LAUNCH(TT, 4); break; \
        default: CFM16_LAUNCH(TT, 8); break; \
    }
        if (dtype == FEN_BF16) {
            CFM16_MB(bf16);
        } else {
            CFM16_MB(f16);
        }
#undef CFM16_MB
#undef CFM16_LAUNCH
        FEN_CHECK_LAUNCH();
        return FEN_OK;
    }
    if (W % 4 == 0) {
        const unsigned nb = (unsigned)((size_t)B * ((H + 1) / 2) * ((W + CF4_TW - 1) / CF4_TW));
        const size_t lds4 = lds + (size_t)Ci * 4 * (CF4_TW + 2) * sizeof(float);
        if (dtype == FEN_BF16)
            hipLaunchKernelGGL(k_conv_first4<bf16>, dim3(nb), dim3(256), lds4, STREAM, B, Ci, H, W, C, x, w, bias,
                               (bf16*)y, in_mean, in_istd, act);
        else if (dtype == FEN_F16)
            hipLaunchKernelGGL(k_conv_first4<f16>, dim3(nb), dim3(256), lds4, STREAM, B, Ci, H, W, C, x, w, bias,
                               (f16*)y, in_mean, in_istd, act);
        else if (dtype == FEN_F32)
            hipLaunchKernelGGL(k_conv_first4<float>, dim3(nb), dim3(256), lds4, STREAM, B, Ci, H, W, C, x, w, bias,
                               (float*)y, in_mean, in_istd, act);
        else
            return FEN_EINVAL;
        FEN_CHECK_LAUNCH();
        return FEN_OK;
    }
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_conv_first<bf16>, dim3(nblk(n)), dim3(256), lds, STREAM, B, Ci, H, W, C, x, w, bias,
                           (bf16*)y, in_mean, in_istd, act);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_conv_first<f16>, dim3(nblk(n)), dim3(256), lds, STREAM, B, Ci, H, W, C, x, w, bias,
                           (f16*)y, in_mean, in_istd, act);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_conv_first<float>, dim3(nblk(n)), dim3(256), lds, STREAM, B, Ci, H, W, C, x, w, bias,
                           (float*)y, in_mean, in_istd, act);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_conv_first_fwd(int dtype, int B, int Ci, int H, int W, int C, const float* x, const float* w,
                                  const float* bias, void* y, void* stream) {
    return fen_conv_first_fwd_ex(dtype, B, Ci, H, W, C, x, w, bias, nullptr, nullptr, -1.f, y, stream);
}

extern "C" size_t fen_conv_first_work_floats(int B, int Ci, int H, int W, int C) {
    return (size_t)CF_BLOCKS * 28 * C;               // one partial row set per block
}

extern "C" int fen_conv_first_wgrad(int dtype, int B, int Ci, int H, int W, int C, const float* x, const void* dy,
                                    float* dw, float* db, int accumulate, float* work, void* stream) {
    if (!x || !dy || !dw || !work || Ci > 3 || C > 128 || B <= 0) return FEN_EINVAL;
    if (C % 16 == 0) {   // (the VALU form below: 223 vs ~70 us at 256x256, B=32; kept for odd C)
        // matrix-core form: MB = 16-channel blocks (C = 32, 64 or 128 on the path)
        auto go = [&](auto tag, auto mb) {
            using TT = decltype(tag);
            constexpr int MBv = decltype(mb)::value;
            hipLaunchKernelGGL((k_conv_first_wgrad_m<TT, MBv>), dim3(CF_BLOCKS), dim3(256), 0, STREAM, B, Ci, H, W, C, x,
                               (const TT*)dy, work);
        };
        const int mb = C <= 32 ? 2 : C <= 64 ? 4 : 8;
        if (dtype == FEN_BF16) {
            if (mb == 2) go(bf16{}, std::integral_constant<int, 2>{});
            else if (mb == 4) go(bf16{}, std::integral_constant<int, 4>{});
            else go(bf16{}, std::integral_constant<int, 8>{});
        } else if (dtype == FEN_F16) {
            if (mb == 2) go(f16{}, std::integral_constant<int, 2>{});
            else if (mb == 4) go(f16{}, std::integral_constant<int, 4>{});
            else go(f16{}, std::integral_constant<int, 8>{});
        } else if (dtype == FEN_F32) {
            if (mb == 2) go(float{}, std::integral_constant<int, 2>{});
            else if (mb == 4) go(float{}, std::integral_constant<int, 4>{});
            else go(float{}, std::integral_constant<int, 8>{});
        } else {
            return FEN_EINVAL;
        }
        FEN_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_conv_first_finalize, dim3(28), dim3(1024), 0, STREAM, CF_BLOCKS, Ci, C, work,
                           dw, db, accumulate);
        FEN_CHECK_LAUNCH();
        return FEN_OK;
    }
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_conv_first_wgrad<bf16>, dim3(CF_BLOCKS), dim3(256), 0, STREAM, B, Ci, H, W, C, x,
                           (const bf16*)dy, work);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_conv_first_wgrad<f16>, dim3(CF_BLOCKS), dim3(256), 0, STREAM, B, Ci, H, W, C, x,
                           (const f16*)dy, work);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_conv_first_wgrad<float>, dim3(CF_BLOCKS), dim3(256), 0, STREAM, B, Ci, H, W, C, x,
                           (const float*)dy, work);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_conv_first_finalize, dim3(28), dim3(1024), 0, STREAM, CF_BLOCKS, Ci, C, work, dw, db,
                       accumulate);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_conv_last_dgrad_part_rows(int B, int H, int W) {
    const size_t ntiles = (size_t)B * ((H + 15) / 16) * ((W + 15) / 16);
    return ntiles < (size_t)CLD_GRID ? ntiles : (size_t)CLD_GRID;     // one partial row per block
}

extern "C" int fen_conv_last_bwd_supported(int dtype, int B, int H, int W, int C, int Co) {
    return (dtype == FEN_BF16 || dtype == FEN_F16) && B > 0 && C == 64 && Co >= 1 && Co <= 3 && H > 0 && W > 0 &&
           H % 16 == 0 && W % 16 == 0;
}

extern "C" int fen_conv_last_bwd(int dtype, int B, int H, int W, int C, int Co, const void* dout, const float* w,
                                 const void* pre, const void* post, const float* alpha, void* du, float* dal_part,
                                 float* dw_part, float* db_part, void* stream) {
    if (!dout || !w || !pre || !post || !alpha || !du || !dal_part || !dw_part || !db_part) return FEN_EINVAL;
    if (!fen_conv_last_bwd_supported(dtype, B, H, W, C, Co)) return FEN_EUNSUPPORTED;
    const int nb = (int)fen_conv_last_dgrad_part_rows(B, H, W);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_cl_bwd<bf16>, dim3(nb), dim3(256), 0, STREAM, B, H, W, Co, (const bf16*)dout, w,
                           (const bf16*)pre, (const bf16*)post, alpha, (bf16*)du, dal_part, dw_part, db_part);
    else
        hipLaunchKernelGGL(k_cl_bwd<f16>, dim3(nb), dim3(256), 0, STREAM, B, H, W, Co, (const f16*)dout, w,
                           (const f16*)pre, (const f16*)post, alpha, (f16*)du, dal_part, dw_part, db_part);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_conv_last_dgrad(int dtype, int B, int H, int W, int C, int Co, const void* dout, const float* w,
                                   const void* pre, const void* post, const float* alpha, void* du, float* part,
                                   void* stream) {
    if (!dout || !w || !pre || !alpha || !du || !part || Co > 3 || C < 32 || C > 256 || 256 % (C / 2) || (H | W) & 1)
        return FEN_EINVAL;
    const int nb = (int)fen_conv_last_dgrad_part_rows(B, H, W);
    auto launch = [&](auto tag) -> int {
        using T = decltype(tag);
        if constexpr (sizeof(T) == 2) {
            if (C == 64 && H % 16 == 0 && W % 16 == 0) {
                hipLaunchKernelGGL((k_cld_p<T>), dim3(nb), dim3(256), 0, STREAM, B, H, W, Co, (const T*)dout, w,
                                   (const T*)pre, (const T*)post, alpha, (T*)du, part);
                return FEN_OK;
            }
        }
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, STREAM, B, H, W, Co, (const T*)dout, w, (const T*)pre,
                               (const T*)post, alpha, (T*)du, part);
        };
        switch (C) {
            case 32: go(k_conv_last_dgrad<T, 32>); break;
            case 64: go(k_conv_last_dgrad<T, 64>); break;
            case 128: go(k_conv_last_dgrad<T, 128>); break;
            case 256: go(k_conv_last_dgrad<T, 256>); break;
            default: return FEN_EINVAL;
        }
        return FEN_OK;
    };
    int rc;
    if (dtype == FEN_BF16) rc = launch(bf16{});
    else if (dtype == FEN_F16) rc = launch(f16{});
    else if (dtype == FEN_F32) rc = launch(0.f);
    else return FEN_EINVAL;
    if (rc != FEN_OK) return rc;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

static bool se_shape_ok(int C, int Cr) { return C > 0 && C <= 256 && C % 16 == 0 && Cr > 0 && Cr <= 64 && Cr % 4 == 0; }

extern "C" int fen_se_fwd(int B, int C, int Cr, int nparts, float inv_hw, const float* part, const float* w1,
                          const float* w2, float* mean, float* hid, float* s, void* stream) {
    if (!part || !w1 || !w2 || !s || B <= 0 || nparts <= 0) return FEN_EINVAL;
    if (!se_shape_ok(C, Cr)) return FEN_EUNSUPPORTED;
    hipLaunchKernelGGL(k_se_fwd, dim3(B), dim3(256), 0, STREAM, C, Cr, nparts, inv_hw, part, w1, w2, mean, hid, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_se_apply(int dtype, int B, int HW, int C, const void* t, const float* s, float res_scale,
                            const void* x, void* y, void* stream) {
    if (!t || !s || !x || !y) return FEN_EINVAL;
    const int V = dtype == FEN_F32 ? 4 : 8;
    if (C % V) return FEN_EUNSUPPORTED;
    const size_t nvec = (size_t)B * HW * C / V;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_apply<bf16, false>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const bf16*)t, s, res_scale, x, (bf16*)y);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL((k_se_apply<f16, false>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const f16*)t, s, res_scale, x, (f16*)y);
    else
        hipLaunchKernelGGL((k_se_apply<float, false>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const float*)t, s, res_scale, x, (float*)y);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_se_fused(int dtype, int B, int HW, int C, int Cr, int nparts, float inv_hw, const float* part,
                            const float* w1, const float* w2, float* mean, float* hid, float* s, const void* t,
                            float res_scale, const void* x, void* y, void* stream) {
    if (!part || !w1 || !w2 || !t || !x || !y || B <= 0 || HW <= 0 || nparts <= 0) return FEN_EINVAL;
    if (!se_shape_ok(C, Cr) || C * Cr > 4096) return FEN_EUNSUPPORTED;
    const int V = dtype == FEN_F32 ? 4 : 8;
    const size_t nv = (size_t)HW * C / V;
    // 8 vectors per thread: 16 blocks per 64x64x64 bf16 image -> 512 blocks at B = 32
    constexpr int NPT = 8;
    const unsigned splits = (unsigned)((nv + 256 * NPT - 1) / (256 * NPT));
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_fused<bf16, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           part, w1, w2, mean, hid, s, (const bf16*)t, res_scale, (const bf16*)x, (bf16*)y);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL((k_se_fused<f16, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           part, w1, w2, mean, hid, s, (const f16*)t, res_scale, (const f16*)x, (f16*)y);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL((k_se_fused<float, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           part, w1, w2, mean, hid, s, (const float*)t, res_scale, (const float*)x, (float*)y);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// pixels per pool_dot block: 64 (HW = 4096 -> 64 chunks x B images = 2048 blocks, ~32 waves
// per CU in flight; 256 px per block left 8 waves per CU and measured 11.7 us per SE backward
// pool inside the training step)
#ifndef POOL_PIX
#define POOL_PIX 64
#endif
extern "C" size_t fen_pool_parts(int HW) {
    int n = HW / POOL_PIX;
    if (n < 1) n = 1;
    if (n > 64) n = 64;
    return (size_t)n;
}

extern "C" int fen_pool_dot(int dtype, int B, int HW, int C, const void* a, const void* b_, float* part,
                            void* stream) {
    const int V = dtype == FEN_F32 ? 4 : 8;
    if (!a || !part || C % V || C / V > 256) return FEN_EINVAL;
    const int nchunk = (int)fen_pool_parts(HW);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_pool_dot<bf16>, dim3(nchunk, B), dim3(256), 0, STREAM, HW, C, nchunk, (const bf16*)a,
                           (const bf16*)b_, part);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_pool_dot<f16>, dim3(nchunk, B), dim3(256), 0, STREAM, HW, C, nchunk, (const f16*)a,
                           (const f16*)b_, part);
    else
        hipLaunchKernelGGL(k_pool_dot<float>, dim3(nchunk, B), dim3(256), 0, STREAM, HW, C, nchunk, (const float*)a,
                           (const float*)b_, part);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_se_bwd(int B, int C, int Cr, int nparts, float inv_hw, float res_scale, const float* part,
                          const float* mean, const float* hid, const float* s, const float* w1, const float* w2,
                          float* g, float* dw1p, float* dw2p, void* stream) {
    if (!part || !mean || !hid || !s || !w1 || !w2 || !g || !dw1p || !dw2p || C > 512 || Cr > 128) return FEN_EINVAL;
    if (C * Cr <= SE_STAGE_MAX)
        hipLaunchKernelGGL(k_se_bwd<true>, dim3(B), dim3(256), 0, STREAM, C, Cr, nparts, inv_hw, res_scale, part, mean,
                           hid, s, w1, w2, g, dw1p, dw2p);
    else
        hipLaunchKernelGGL(k_se_bwd<false>, dim3(B), dim3(256), 0, STREAM, C, Cr, nparts, inv_hw, res_scale, part, mean,
                           hid, s, w1, w2, g, dw1p, dw2p);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_se_bwd_apply(int dtype, int B, int HW, int C, const void* dy, const float* s, float res_scale,
                                const float* g, void* dt, void* stream) {
    if (!dy || !s || !g || !dt) return FEN_EINVAL;
    const int V = dtype == FEN_F32 ? 4 : 8;
    if (C % V) return FEN_EUNSUPPORTED;
    const size_t nvec = (size_t)B * HW * C / V;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_apply<bf16, true>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const bf16*)dy, s, res_scale, (const void*)g, (bf16*)dt);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL((k_se_apply<f16, true>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const f16*)dy, s, res_scale, (const void*)g, (f16*)dt);
    else
        hipLaunchKernelGGL((k_se_apply<float, true>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const float*)dy, s, res_scale, (const void*)g, (float*)dt);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_se_bwd_fused(int dtype, int B, int HW, int C, int Cr, int nparts, float inv_hw, float res_scale,
                                const float* part, const float* mean, const float* hid, const float* s,
                                const float* w1, const float* w2, const void* dy, float* g, float* dw1p, float* dw2p,
                                void* dt, void* stream) {
    if (!part || !mean || !hid || !s || !w1 || !w2 || !dy || !dw1p || !dw2p || !dt || B <= 0 || HW <= 0)
        return FEN_EINVAL;
    const int V = dtype == FEN_F32 ? 4 : 8;
    if (C <= 0 || C > 64 || C % V || Cr <= 0 || Cr > 64 || C * Cr > 4096 || (C * Cr) % 4 || nparts <= 0 || nparts > 64)
        return FEN_EUNSUPPORTED;
    const size_t nv = (size_t)HW * C / V;
    constexpr int NPT = 8;
    const unsigned splits = (unsigned)((nv + 256 * NPT - 1) / (256 * NPT));
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_bwd_fused<bf16, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           res_scale, part, mean, hid, s, w1, w2, (const bf16*)dy, g, dw1p, dw2p, (bf16*)dt);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL((k_se_bwd_fused<f16, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           res_scale, part, mean, hid, s, w1, w2, (const f16*)dy, g, dw1p, dw2p, (f16*)dt);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL((k_se_bwd_fused<float, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts,
                           inv_hw, res_scale, part, mean, hid, s, w1, w2, (const float*)dy, g, dw1p, dw2p, (float*)dt);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_bicubic_down4(int B, int C, int H, int W, const float* hr, float* lr, void* stream) {
    if (!hr || !lr || H < 4 || W < 4) return FEN_EINVAL;
    const size_t n = (size_t)B * C * (H / 4) * (W / 4);
    hipLaunchKernelGGL(k_bicubic_down4, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, hr, lr);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_colsum_multi(int njobs, const fen_colsum_job* jobs, void* stream) {
    if (njobs <= 0 || njobs > COLSUM_MAXJ || !jobs) return FEN_EINVAL;
    ColJobs k;
    k.n = njobs;
    int blk = 0, slot = 0;
    for (int i = 0; i < njobs; ++i) {
        const fen_colsum_job& j = jobs[i];
        if (!j.part || !j.out || j.rows <= 0 || j.cols <= 0) return FEN_EINVAL;
        const int ncb = (j.cols + 63) / 64;
        // tall narrow jobs (conv_last's 8192 x 64 slope rows at B=32): up to 8 row slices of
        // >= 512 rows.  At 2048 rows (the strip backward's, 10 per launch) a split measured
        // 12.3 vs 11.2 us per launch: the split's combine costs more than the round trips saved
        int ns = 1;
        if (j.cols > 1 && ncb <= 2 && j.rows >= 4096 && slot + ncb <= COLSUM_SLOTS) ns = j.rows / 512 < 8 ? j.rows / 512 : 8;
        k.j[i] = ColJobK{j.part, j.out, j.rows, j.cols, j.scale, j.accumulate, blk, ns, slot};
        if (ns > 1) slot += ncb;
        blk += j.cols == 1 ? 1 : ncb * ns;
    }
    hipLaunchKernelGGL(k_colsum_multi, dim3(blk), dim3(1024), 0, STREAM, k);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_colsum(int rows, int cols, const float* part, float scale, float* out, int accumulate,
                          void* stream) {
    const fen_colsum_job j{part, out, rows, cols, scale, accumulate};
    return fen_colsum_multi(1, &j, stream);
}

extern "C" size_t fen_packed_elems(int mode, int Cout, int Cin) {
    if (mode == 2) return (size_t)9 * ((Cin + 15) & ~15) * Cout;
    return (size_t)9 * ((Cout + 15) & ~15) * Cin;
}

extern "C" int fen_pack_conv_w(int dtype, int mode, int Cout, int Cin, const float* w, void* out, void* stream) {
    if (!w || !out || mode < 0 || mode > 2 || (mode == 1 && Cout % 4)) return FEN_EINVAL;
    const size_t n = fen_packed_elems(mode, Cout, Cin);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_pack<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, mode, Cout, Cin, w, (bf16*)out, n);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_pack<f16>, dim3(nblk(n)), dim3(256), 0, STREAM, mode, Cout, Cin, w, (f16*)out, n);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_pack<float>, dim3(nblk(n)), dim3(256), 0, STREAM, mode, Cout, Cin, w, (float*)out, n);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_pack_table_bytes(int njobs) {
    return (size_t)njobs * (sizeof(PackJobK) + sizeof(unsigned long long)) + sizeof(unsigned long long);
}

extern "C" int fen_pack_table(int dtype, int njobs, const fen_pack_job* jobs, void* table_host, size_t* total) {
    if (njobs <= 0 || !jobs || !table_host || !total || (dtype != FEN_BF16 && dtype != FEN_F16 && dtype != FEN_F32)) return FEN_EINVAL;
    PackJobK* pj = (PackJobK*)table_host;
    unsigned long long* e0 = (unsigned long long*)(pj + njobs);
    unsigned long long acc = 0;
    for (int i = 0; i < njobs; ++i) {
        const fen_pack_job& j = jobs[i];
        if (!j.w || !j.out || j.mode < 0 || j.mode > 2 || (j.mode == 1 && j.Cout % 4)) return FEN_EINVAL;
        const size_t n = fen_packed_elems(j.mode, j.Cout, j.Cin);
        if (n >= (1ull << 31) || n % PACK_RUN) return FEN_EUNSUPPORTED;
        pj[i] = PackJobK{j.w, j.out, j.mode, j.Cout, j.Cin, (unsigned)n};
        e0[i] = acc;
        acc += (n + PACK_BLK - 1) / PACK_BLK * PACK_BLK;
    }
    e0[njobs] = acc;
    *total = (size_t)acc;
    return FEN_OK;
}

extern "C" int fen_pack_multi(int dtype, int njobs, const void* table_dev, size_t total, void* stream) {
    if (njobs <= 0 || !table_dev || total == 0) return FEN_EINVAL;
    const PackJobK* pj = (const PackJobK*)table_dev;
    const unsigned long long* e0 = (const unsigned long long*)(pj + njobs);
    const unsigned nb = (unsigned)((total + PACK_BLK - 1) / PACK_BLK);   // 256 threads x PACK_RUN
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_pack_multi<bf16>, dim3(nb), dim3(256), 0, STREAM, njobs, pj, e0, (unsigned long long)total);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_pack_multi<f16>, dim3(nb), dim3(256), 0, STREAM, njobs, pj, e0, (unsigned long long)total);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_pack_multi<float>, dim3(nb), dim3(256), 0, STREAM, njobs, pj, e0, (unsigned long long)total);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_nchw_to_nhwc(int dtype, int B, int C, int H, int W, int Cpad, const float* x, void* y,
                                void* stream) {
    if (!x || !y || Cpad < C) return FEN_EINVAL;
    const size_t n = (size_t)B * Cpad * H * W;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_nchw_to_nhwc<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, Cpad, x, (bf16*)y);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_nchw_to_nhwc<f16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, Cpad, x, (f16*)y);
    else
        hipLaunchKernelGGL(k_nchw_to_nhwc<float>, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, Cpad, x, (float*)y);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_prelu_bwd_unshuffle(int dtype, int B, int H, int W, int C, const void* dy, const void* pre,
                                       const float* alpha, void* du, float* part, void* stream) {
    if (!dy || !pre || !alpha || !du || !part || C < 32 || C > 256 || 256 % (C / 2) || (H | W) & 1)
        return FEN_EINVAL;
    const int nb = B * ((H + 15) / 16) * ((W + 15) / 16);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_prelu_bwd_unshuffle<bf16>, dim3(nb), dim3(256), 0, STREAM, B, H, W, C, (const bf16*)dy,
                           (const bf16*)pre, alpha, (bf16*)du, part);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_prelu_bwd_unshuffle<f16>, dim3(nb), dim3(256), 0, STREAM, B, H, W, C, (const f16*)dy,
                           (const f16*)pre, alpha, (f16*)du, part);
    else
        hipLaunchKernelGGL(k_prelu_bwd_unshuffle<float>, dim3(nb), dim3(256), 0, STREAM, B, H, W, C,
                           (const float*)dy, (const float*)pre, alpha, (float*)du, part);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_nhwc_to_nchw(int dtype, int B, int C, int H, int W, const void* x, float* y, void* stream) {
    if (!x || !y) return FEN_EINVAL;
    const size_t n = (size_t)B * C * H * W;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_nhwc_to_nchw<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, (const bf16*)x, y);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_nhwc_to_nchw<f16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, (const f16*)x, y);
    else
        hipLaunchKernelGGL(k_nhwc_to_nchw<float>, dim3(nblk(n)), dim3(256), 0, STREAM, B, C, H, W, (const float*)x, y);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_sumsq_parts(size_t n) {
    size_t b = (n / 4 + 255) / 256;
    if (b < 1) b = 1;
    if (b > SUMSQ_BLOCKS_MAX) b = SUMSQ_BLOCKS_MAX;
    return (int)b;
}

extern "C" int fen_sumsq(size_t n, const float* g, float* part, void* stream) {
    if (!g || !part || ((uintptr_t)g & 15)) return FEN_EINVAL;
    hipLaunchKernelGGL(k_sumsq, dim3(fen_sumsq_parts(n)), dim3(256), 0, STREAM, n, g, part);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_optim_prepare(int nparts, const float* part, float max_norm, float beta1, float beta2, float wd,
                                 float* scal, void* stream) {
    if (!part || !scal || nparts <= 0) return FEN_EINVAL;
    hipLaunchKernelGGL(k_optim_prepare, dim3(1), dim3(256), 0, STREAM, nparts, part, max_norm, beta1, beta2, wd, scal);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_adamw(size_t n, float* p, const float* g, float* m, float* v, const float* scal, float beta1,
                         float beta2, float eps, void* stream) {
    if (!p || !g || !m || !v || !scal) return FEN_EINVAL;
    hipLaunchKernelGGL(k_adamw, dim3(nblk(n)), dim3(256), 0, STREAM, n, p, g, m, v, scal, beta1, beta2, eps);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_adamw_multi(int njobs, const fen_adamw_job* jobs, float lr, float beta1, float beta2,
                               float one_minus_beta1, float one_minus_beta2, float eps, float weight_decay,
                               void* stream) {
    if (njobs <= 0 || njobs > ADAMW_MAXJ || !jobs) return FEN_EINVAL;
    AdamJobs k;
    k.n = njobs, k.lr = lr, k.b1 = beta1, k.b2 = beta2, k.eps = eps, k.wd = weight_decay;
    k.omb1 = one_minus_beta1, k.omb2 = one_minus_beta2;
    long long blk = 0;
    for (int i = 0; i < njobs; ++i) {
        const fen_adamw_job& j = jobs[i];
        if (!j.p || !j.g || !j.m || !j.v || !j.step || j.n <= 0) return FEN_EINVAL;
        const bool vec = !(((uintptr_t)j.p | (uintptr_t)j.g | (uintptr_t)j.m | (uintptr_t)j.v) & 15);
        k.j[i] = AdamJobK{j.p, j.g, j.m, j.v, j.step, (long long)j.n, (int)blk, vec ? 1 : 0};
        blk += ((long long)j.n + ADAM_BLK - 1) / ADAM_BLK;
        if (blk >= (1ll << 30)) return FEN_EUNSUPPORTED;
    }
    hipLaunchKernelGGL(k_adamw_steps, dim3(1), dim3(64), 0, STREAM, k);
    hipLaunchKernelGGL(k_adamw_multi, dim3((unsigned)blk), dim3(256), 0, STREAM, k);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_scale(size_t n, float* y, float s, void* stream) {
    if (!y) return FEN_EINVAL;
    hipLaunchKernelGGL(k_scale, dim3(nblk(n)), dim3(256), 0, STREAM, n, y, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

namespace fen_detail {
thread_local int last_hip_error = 0;
}

extern "C" const char* fen_last_hip_error(void) {
    const int e = fen_detail::last_hip_error;
    return e ? hipGetErrorString((hipError_t)e) : "none";
}

extern "C" int fen_status_word(void** host, void** dev) {
    if (!host || !dev) return FEN_EINVAL;
    static void* words[64] = {};
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e == hipSuccess && (d < 0 || d >= 64)) return FEN_EUNSUPPORTED;
    if (e == hipSuccess && !words[d]) {
        e = hipHostMalloc(&words[d], 64, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) { for (int i = 0; i < 16; ++i) ((volatile int*)words[d])[i] = 0; }
        else words[d] = nullptr;
    }
    if (e == hipSuccess) e = hipHostGetDevicePointer(dev, words[d], 0);
    if (e != hipSuccess) {
        fen_detail::last_hip_error = (int)e;
        return FEN_EHIP;
    }
    *host = words[d];
    return FEN_OK;
}

extern "C" int fen_status_take(void* host) {
    return host ? __atomic_exchange_n((int*)host, 0, __ATOMIC_ACQ_REL) : 0;
}

extern "C" const char* fen_status_string(int code) {
    switch (code) {
        case FEN_OK: return "FEN_OK";
        case FEN_EINVAL: return "FEN_EINVAL: invalid pointer, shape or alignment";
        case FEN_EUNSUPPORTED: return "FEN_EUNSUPPORTED: configuration not implemented by the gfx950 kernels";
        case FEN_EHIP: return "FEN_EHIP: HIP kernel launch failed";
        case FEN_ERCCL: return "FEN_ERCCL: RCCL call failed";
        default: return "FEN_?: unknown status";
    }
}

extern "C" const char* fen_build_info(void) {
    return "libfen_hip gfx950 (CDNA4) MFMA kernels, built " __DATE__ " " __TIME__;
}

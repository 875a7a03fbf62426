// Bandwidth-bound kernels of the FaceEnhanceNet hot path (gfx950): conv_first (K=27),
// conv_last data-gradient (K=27) fused with PReLU backward + PixelShuffle inverse, the
// channel-attention (SE) forward/backward pieces, the bicubic /4 LR synthesis, weight
// packing, deterministic column reductions and the fused clip_grad_norm_ + AdamW.
// All vector accesses are 16 B per lane.
#include "fen_common.h"

namespace {

inline int nblk(size_t n, int t = 256) { return (int)((n + t - 1) / t); }

// ------------------------------ conv_first (3 -> C) ------------------------------
// reference custom.py:91-94,164; thread per (pixel, 8 output channels)
template <typename T>
__global__ void k_conv_first(int B, int Ci, int H, int W, int C, const float* __restrict__ x,
                             const float* __restrict__ w, const float* __restrict__ bias, T* __restrict__ y) {
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
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int hh = hq + t / 3 - 1, ww = wq + t % 3 - 1;
            const float v = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) ? xp[(size_t)hh * W + ww] : 0.f;
            const float4* wp = (const float4*)(sw + (ci * 9 + t) * C + g * 8);
            const float4 w0 = wp[0], w1 = wp[1];
            acc[0] += v * w0.x; acc[1] += v * w0.y; acc[2] += v * w0.z; acc[3] += v * w0.w;
            acc[4] += v * w1.x; acc[5] += v * w1.y; acc[6] += v * w1.z; acc[7] += v * w1.w;
        }
    }
    char* o = (char*)y + (px * C + g * 8) * sizeof(T);
    if constexpr (sizeof(T) == 2) {
        *(uint4*)o = pack16<bf16>(acc);
    } else {
        *(uint4*)o = pack16<float>(acc);
        *(uint4*)(o + 16) = pack16<float>(acc + 4);
    }
}

// conv_first weight gradient: wave = one pixel at a time (uniform x loads), lane = co
constexpr int CF_BLOCKS = 512;
template <typename T>
__global__ __launch_bounds__(256) void k_conv_first_wgrad(int B, int Ci, int H, int W, int C, const float* __restrict__ x,
                                   const T* __restrict__ dy, float* __restrict__ part) {
    __shared__ float red[4][28 * 2][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float acc[2][28];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int k = 0; k < 28; ++k) acc[j][k] = 0.f;
    const size_t npx = (size_t)B * H * W;
    const int nc = (C + 63) / 64;
    for (size_t px = (size_t)blockIdx.x * 4 + wave; px < npx; px += (size_t)gridDim.x * 4) {
        const size_t pu = __builtin_amdgcn_readfirstlane((unsigned)px);
        const int wq = (int)(pu % W), hq = (int)((pu / W) % H), b = (int)(pu / ((size_t)W * H));
        float g[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int co = lane + 64 * j;
            g[j] = (j < nc && co < C) ? tof<T>(dy[pu * C + co]) : 0.f;
        }
        for (int ci = 0; ci < Ci; ++ci) {
            const float* xp = x + ((size_t)b * Ci + ci) * H * W;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int hh = hq + t / 3 - 1, ww = wq + t % 3 - 1;
                const float v = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) ? xp[(size_t)hh * W + ww] : 0.f;
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j][ci * 9 + t] += g[j] * v;
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j][27] += g[j];
    }
    for (int j = 0; j < nc; ++j)
        for (int k = 0; k < 28; ++k) red[wave][j * 28 + k][lane] = acc[j][k];
    __syncthreads();
    for (int i = threadIdx.x; i < nc * 28 * 64; i += 256) {
        const int lanei = i & 63, jk = i >> 6;
        const float s = red[0][jk][lanei] + red[1][jk][lanei] + red[2][jk][lanei] + red[3][jk][lanei];
        const int j = jk / 28, k = jk % 28, co = lanei + 64 * j;
        if (co < C) part[((size_t)blockIdx.x * 28 + k) * C + co] = s;
    }
}

__global__ void k_conv_first_finalize(int nb, int Ci, int C, const float* part, float* dw, float* db, int accum) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // over 28*C
    if (i >= 28 * C) return;
    const int k = i / C, co = i % C;
    if (k >= Ci * 9 && k != 27) return;
    float s = 0.f;
    for (int r = 0; r < nb; ++r) s += part[((size_t)r * 28 + k) * C + co];
    if (k == 27) {
        if (db) db[co] = accum ? db[co] + s : s;
    } else {
        float* o = dw + (size_t)co * Ci * 9 + k;
        *o = accum ? *o + s : s;
    }
}

// --------------- conv_last dgrad + PReLU backward + PixelShuffle inverse ---------------
// dout NHWC16 [B,H,W,16], w [Co][C][3][3] -> da[px][c] -> dv = da*(pre>0?1:alpha[c])
// -> du[b][h/2][w/2][4c + 2(h&1) + (w&1)];  block = 16x16 source px = 8x8 du px
template <typename T>
__global__ __launch_bounds__(256) void k_conv_last_dgrad(int B, int H, int W, int C, int Co, const T* __restrict__ dout,
                                  const float* __restrict__ w, const T* __restrict__ pre,
                                  const float* __restrict__ alpha, T* __restrict__ du, float* __restrict__ part) {
    __shared__ float4 sd[18 * 18];          // dout tile + halo, channels 0..2 (3 = pad)
    __shared__ float sdal[256 * 2];
    const int tid = threadIdx.x;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int b = blockIdx.x / tpi, tile = blockIdx.x - b * tpi;
    const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
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
    const int K2 = C / 2;
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
    __syncthreads();
    float dal0 = 0.f, dal1 = 0.f;
    const int Hh = H >> 1, Wh = W >> 1;
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
            const size_t pi = ((size_t)(b * H + h0 + sh) * W + w0 + sw) * C + 2 * k;
            const float p0 = tof<T>(pre[pi]), p1 = tof<T>(pre[pi + 1]);
            dal0 += p0 > 0.f ? 0.f : da0 * p0;
            dal1 += p1 > 0.f ? 0.f : da1 * p1;
            out[t] = p0 > 0.f ? da0 : da0 * al0;
            out[4 + t] = p1 > 0.f ? da1 : da1 * al1;
        }
        char* o = (char*)du + (((size_t)(b * Hh + gh2) * Wh + gw2) * (4 * C) + 8 * k) * sizeof(T);
        if constexpr (sizeof(T) == 2) {
            *(uint4*)o = pack16<bf16>(out);
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
// (a few KB of L2 reads), block 0 of each image stores mean/hid/s.  Each thread issues the
// loads of its NPT t / x vectors BEFORE the gate, so the gate's latency hides under them,
// then writes y = t * s[c] * rs + x.
template <typename T, int NPT>
__global__ __launch_bounds__(256) void k_se_fused(int HW, int C, int Cr, int nparts, float inv_hw,
                                                  const float* __restrict__ part, const float* __restrict__ w1,
                                                  const float* __restrict__ w2, float* mean, float* hid, float* s,
                                                  const T* __restrict__ t, float rs, const T* __restrict__ x,
                                                  T* __restrict__ y) {
    __shared__ float sm[256], sh[64], sg[256], red[256];
    constexpr int V = 16 / sizeof(T);
    const int b = blockIdx.y;
    const size_t nv = (size_t)HW * C / V;
    const size_t base = (size_t)b * nv;
    const size_t v0 = (size_t)blockIdx.x * (256 * NPT) + threadIdx.x;
    uint4 tv[NPT], xv[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const size_t v = v0 + (size_t)j * 256;
        if (v < nv) {
            tv[j] = *(const uint4*)(t + (base + v) * V);
            xv[j] = *(const uint4*)(x + (base + v) * V);
        }
    }
    const bool first = blockIdx.x == 0;
    se_gate(b, C, Cr, nparts, inv_hw, part, w1, w2, sm, sh, sg, red, first ? mean : nullptr,
            first ? hid : nullptr, first ? s : nullptr);
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const size_t v = v0 + (size_t)j * 256;
        if (v < nv) {
            const int c0 = (int)((v * V) % C);
            float a[V], bb[V], o[V];
            unpack16<T>(tv[j], a);
            unpack16<T>(xv[j], bb);
#pragma unroll
            for (int k = 0; k < V; ++k) o[k] = a[k] * sg[c0 + k] * rs + bb[k];
            *(uint4*)(y + (base + v) * V) = pack16<T>(o);
        }
    }
}

extern "C" int fen_conv_first_fwd(int dtype, int B, int Ci, int H, int W, int C, const float* x, const float* w,
                                  const float* bias, void* y, void* stream) {
    if (!x || !w || !bias || !y || B <= 0 || Ci <= 0 || Ci > 3 || C % 8 || C > 128) return FEN_EINVAL;
    const size_t n = (size_t)B * H * W * (C / 8);
    const size_t lds = (size_t)Ci * 9 * C * sizeof(float);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_conv_first<bf16>, dim3(nblk(n)), dim3(256), lds, STREAM, B, Ci, H, W, C, x, w, bias, (bf16*)y);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_conv_first<float>, dim3(nblk(n)), dim3(256), lds, STREAM, B, Ci, H, W, C, x, w, bias, (float*)y);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_conv_first_work_floats(int B, int Ci, int H, int W, int C) {
    return (size_t)CF_BLOCKS * 28 * C;
}

extern "C" int fen_conv_first_wgrad(int dtype, int B, int Ci, int H, int W, int C, const float* x, const void* dy,
                                    float* dw, float* db, int accumulate, float* work, void* stream) {
    if (!x || !dy || !dw || !work || Ci > 3 || C > 128 || B <= 0) return FEN_EINVAL;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_conv_first_wgrad<bf16>, dim3(CF_BLOCKS), dim3(256), 0, STREAM, B, Ci, H, W, C, x,
                           (const bf16*)dy, work);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_conv_first_wgrad<float>, dim3(CF_BLOCKS), dim3(256), 0, STREAM, B, Ci, H, W, C, x,
                           (const float*)dy, work);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_conv_first_finalize, dim3(nblk(28 * C)), dim3(256), 0, STREAM, CF_BLOCKS, Ci, C, work, dw,
                       db, accumulate);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_conv_last_dgrad_part_rows(int B, int H, int W) {
    return (size_t)B * ((H + 15) / 16) * ((W + 15) / 16);
}

extern "C" int fen_conv_last_dgrad(int dtype, int B, int H, int W, int C, int Co, const void* dout, const float* w,
                                   const void* pre, const float* alpha, void* du, float* part, void* stream) {
    if (!dout || !w || !pre || !alpha || !du || !part || Co > 3 || C < 32 || C > 256 || 256 % (C / 2) || (H | W) & 1)
        return FEN_EINVAL;
    const int nb = (int)fen_conv_last_dgrad_part_rows(B, H, W);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_conv_last_dgrad<bf16>, dim3(nb), dim3(256), 0, STREAM, B, H, W, C, Co, (const bf16*)dout,
                           w, (const bf16*)pre, alpha, (bf16*)du, part);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_conv_last_dgrad<float>, dim3(nb), dim3(256), 0, STREAM, B, H, W, C, Co,
                           (const float*)dout, w, (const float*)pre, alpha, (float*)du, part);
    else
        return FEN_EINVAL;
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
    const int V = dtype == FEN_BF16 ? 8 : 4;
    if (C % V) return FEN_EUNSUPPORTED;
    const size_t nvec = (size_t)B * HW * C / V;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_apply<bf16, false>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const bf16*)t, s, res_scale, x, (bf16*)y);
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
    if (!se_shape_ok(C, Cr)) return FEN_EUNSUPPORTED;
    const int V = dtype == FEN_BF16 ? 8 : 4;
    const size_t nv = (size_t)HW * C / V;
    // 8 vectors per thread: 16 blocks per 64x64x64 bf16 image -> 512 blocks at B = 32
    constexpr int NPT = 8;
    const unsigned splits = (unsigned)((nv + 256 * NPT - 1) / (256 * NPT));
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_fused<bf16, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           part, w1, w2, mean, hid, s, (const bf16*)t, res_scale, (const bf16*)x, (bf16*)y);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL((k_se_fused<float, NPT>), dim3(splits, B), dim3(256), 0, STREAM, HW, C, Cr, nparts, inv_hw,
                           part, w1, w2, mean, hid, s, (const float*)t, res_scale, (const float*)x, (float*)y);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" size_t fen_pool_parts(int HW) {
    int n = HW / 256;
    if (n < 1) n = 1;
    if (n > 64) n = 64;
    return (size_t)n;
}

extern "C" int fen_pool_dot(int dtype, int B, int HW, int C, const void* a, const void* b_, float* part,
                            void* stream) {
    const int V = dtype == FEN_BF16 ? 8 : 4;
    if (!a || !part || C % V || C / V > 256) return FEN_EINVAL;
    const int nchunk = (int)fen_pool_parts(HW);
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_pool_dot<bf16>, dim3(nchunk, B), dim3(256), 0, STREAM, HW, C, nchunk, (const bf16*)a,
                           (const bf16*)b_, part);
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
    hipLaunchKernelGGL(k_se_bwd, dim3(B), dim3(256), 0, STREAM, C, Cr, nparts, inv_hw, res_scale, part, mean, hid, s,
                       w1, w2, g, dw1p, dw2p);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_se_bwd_apply(int dtype, int B, int HW, int C, const void* dy, const float* s, float res_scale,
                                const float* g, void* dt, void* stream) {
    if (!dy || !s || !g || !dt) return FEN_EINVAL;
    const int V = dtype == FEN_BF16 ? 8 : 4;
    if (C % V) return FEN_EUNSUPPORTED;
    const size_t nvec = (size_t)B * HW * C / V;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL((k_se_apply<bf16, true>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const bf16*)dy, s, res_scale, (const void*)g, (bf16*)dt);
    else
        hipLaunchKernelGGL((k_se_apply<float, true>), dim3(nblk(nvec)), dim3(256), 0, STREAM, nvec, HW, C,
                           (const float*)dy, s, res_scale, (const void*)g, (float*)dt);
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

extern "C" int fen_colsum(int rows, int cols, const float* part, float scale, float* out, int accumulate,
                          void* stream) {
    if (!part || !out || rows <= 0 || cols <= 0) return FEN_EINVAL;
    float* p = const_cast<float*>(part);  // stage 1 reduces in place (documented: part is clobbered)
    hipLaunchKernelGGL(k_colsum1, dim3((cols + 63) / 64, (rows + COLSUM_RB - 1) / COLSUM_RB), dim3(256), 0, STREAM,
                       rows, cols, p);
    FEN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_colsum2, dim3(nblk(cols)), dim3(256), 0, STREAM, rows, cols, (const float*)p, scale, out,
                       accumulate);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
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
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_pack<float>, dim3(nblk(n)), dim3(256), 0, STREAM, mode, Cout, Cin, w, (float*)out, n);
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

extern "C" int fen_scale(size_t n, float* y, float s, void* stream) {
    if (!y) return FEN_EINVAL;
    hipLaunchKernelGGL(k_scale, dim3(nblk(n)), dim3(256), 0, STREAM, n, y, s);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" const char* fen_status_string(int code) {
    switch (code) {
        case FEN_OK: return "FEN_OK";
        case FEN_EINVAL: return "FEN_EINVAL: invalid pointer, shape or alignment";
        case FEN_EUNSUPPORTED: return "FEN_EUNSUPPORTED: configuration not implemented by the gfx950 kernels";
        case FEN_EHIP: return "FEN_EHIP: HIP kernel launch failed";
        default: return "FEN_?: unknown status";
    }
}

extern "C" const char* fen_build_info(void) {
    return "libfen_hip gfx950 (CDNA4) MFMA kernels, built " __DATE__ " " __TIME__;
}

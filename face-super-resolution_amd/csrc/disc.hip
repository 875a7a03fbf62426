// VGG-style discriminator pieces (reference src/models/discriminator.py:12-219) that the
// conv kernels do not cover: train-mode BatchNorm2d (+ the LeakyReLU(0.2) that follows it,
// discriminator.py:47-55) forward / backward with running-statistics update, and the
// stride-2 helpers (a stride-2 3x3 conv = the stride-1 conv at full resolution, subsampled;
// its data/weight gradients = the stride-1 ones of the zero-inserted output gradient).
// NHWC activations of the compute dtype; statistics and reductions in fp32 with a per-channel
// shift (the channel's first value) against cancellation; fixed-order partials: deterministic.
#include "fen_common.h"

namespace {

inline int nblk(size_t n, int t = 256) { return (int)((n + t - 1) / t); }
constexpr int BN_BLOCKS = 512;

// part[blk][c] = (sum (y - shift_c), sum (y - shift_c)^2) over the block's pixels; thread =
// (pixel lane, 8-channel group)
template <typename T>
__global__ __launch_bounds__(256) void k_bn_stats(size_t npx, int C, const T* __restrict__ y,
                                                  float* __restrict__ part) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;                     // channel groups (C % 8 == 0, C / V <= 256)
    const int lanes = 256 / G > 0 ? 256 / G : 1;
    const int g = threadIdx.x % G, pl = threadIdx.x / G;
    __shared__ float red[2][256][V];
    float s[V], q[V], sh[V];
    unpack16<T>(*(const uint4*)(y + g * V), sh);          // shift = pixel 0's values
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = q[j] = 0.f;
    if (pl < lanes) {
        for (size_t p = (size_t)blockIdx.x * lanes + pl; p < npx; p += (size_t)gridDim.x * lanes) {
            float v[V];
            unpack16<T>(*(const uint4*)(y + p * C + g * V), v);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float d = v[j] - sh[j];
                s[j] += d;
                q[j] += d * d;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) { red[0][threadIdx.x][j] = s[j]; red[1][threadIdx.x][j] = q[j]; }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
        const int gg = c / V, j = c % V;
        float a = 0.f, b = 0.f;
        for (int l = 0; l < lanes; ++l) { a += red[0][l * G + gg][j]; b += red[1][l * G + gg][j]; }
        part[(size_t)blockIdx.x * 2 * C + c] = a;
        part[(size_t)blockIdx.x * 2 * C + C + c] = b;
    }
}

// per channel: mean, rstd (biased var, eps) -> stat[0..C) mean, stat[C..2C) rstd; running
// stats (momentum m, unbiased var) updated when running_mean != NULL
// 64 channels per block, 16 waves each summing every 16th partial (loads in flight across the
// waves; one thread walking all BN_BLOCKS partials took ~130 us), fixed-order combine in LDS
constexpr int FIN_WAVES = 16;
template <typename T>
__global__ __launch_bounds__(64 * FIN_WAVES) void k_bn_finalize(int nblocks, size_t npx, int C, const T* __restrict__ y,
                                                              const float* __restrict__ part, float eps, float momentum,
                                                              float* __restrict__ stat, float* __restrict__ rmean,
                                                              float* __restrict__ rvar) {
    __shared__ double red[2][FIN_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    double s = 0.0, q = 0.0;
    if (c < C) {
        for (int b = w; b < nblocks; b += FIN_WAVES) {
            s += part[(size_t)b * 2 * C + c];
            q += part[(size_t)b * 2 * C + C + c];
        }
    }
    red[0][w][lane] = s;
    red[1][w][lane] = q;
    __syncthreads();
    if (w != 0 || c >= C) return;
    s = 0.0;
    q = 0.0;
    for (int k = 0; k < FIN_WAVES; ++k) {
        s += red[0][k][lane];
        q += red[1][k][lane];
    }
    const double n = (double)npx;
    const double md = s / n;                                  // mean of (y - shift)
    double var = q / n - md * md;
    if (var < 0) var = 0;
    const float mean = (float)(md + (double)tof<T>(y[c]));
    stat[c] = mean;
    stat[C + c] = (float)(1.0 / sqrt(var + (double)eps));
    if (rmean) {
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(var * n / (n > 1 ? n - 1 : 1));
    }
}

// out = lrelu((y - mean) * rstd * gamma + beta, slope); eval mode passes the running stats
// The per-channel operands are staged in LDS once per block (C <= 1024): with them read
// from global memory per element, every 16-B data vector cost 8 more vector-memory
// instructions (L1 hits, but issue-bound: 66 us average per call in the GAN iteration).
// Each thread streams BN_NPT vectors, all loads first; same arithmetic as before.
constexpr int BN_NPT = 4;
template <typename T>
__global__ __launch_bounds__(256) void k_bn_apply(size_t nv, int C, const T* __restrict__ y,
                                                  const float* __restrict__ mean, const float* __restrict__ rstd,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float slope, T* __restrict__ out) {
    constexpr int V = 16 / sizeof(T);
    __shared__ float sm[1024], sr[1024], sg[1024], sb[1024];
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        sm[c] = mean[c];
        sr[c] = rstd[c];
        sg[c] = gamma[c];
        sb[c] = beta[c];
    }
    const size_t i0 = (size_t)blockIdx.x * (256 * BN_NPT) + threadIdx.x;
    uint4 d[BN_NPT];
#pragma unroll
    for (int k = 0; k < BN_NPT; ++k) {
        const size_t i = i0 + (size_t)k * 256;
        if (i < nv) d[k] = *(const uint4*)(y + i * V);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BN_NPT; ++k) {
        const size_t i = i0 + (size_t)k * 256;
        if (i >= nv) break;
        const int c0 = (int)((i * V) % C);
        float v[V];
        unpack16<T>(d[k], v);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int c = c0 + j;
            const float z = (v[j] - sm[c]) * sr[c] * sg[c] + sb[c];
            v[j] = z > 0.f ? z : slope * z;
        }
        *(uint4*)(out + i * V) = pack16<T>(v);
    }
}

// backward partials: dz = da * (z > 0 ? 1 : slope), xh = (y - mean) rstd, z = gamma xh + beta;
// part[blk] = (sum dz, sum dz * xh) per channel
template <typename T>
__global__ __launch_bounds__(256) void k_bn_bwd_reduce(size_t npx, int C, const T* __restrict__ da,
                                                       const T* __restrict__ y, const float* __restrict__ stat,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float slope, float* __restrict__ part) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;
    const int lanes = 256 / G > 0 ? 256 / G : 1;
    const int g = threadIdx.x % G, pl = threadIdx.x / G;
    __shared__ float red[2][256][V];
    float s[V], q[V];
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = q[j] = 0.f;
    if (pl < lanes) {
        for (size_t p = (size_t)blockIdx.x * lanes + pl; p < npx; p += (size_t)gridDim.x * lanes) {
            float dv[V], yv[V];
            unpack16<T>(*(const uint4*)(da + p * C + g * V), dv);
            unpack16<T>(*(const uint4*)(y + p * C + g * V), yv);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int c = g * V + j;
                const float xh = (yv[j] - stat[c]) * stat[C + c];
                const float z = gamma[c] * xh + beta[c];
                const float dz = z > 0.f ? dv[j] : slope * dv[j];
                s[j] += dz;
                q[j] += dz * xh;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) { red[0][threadIdx.x][j] = s[j]; red[1][threadIdx.x][j] = q[j]; }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
        const int gg = c / V, j = c % V;
        float a = 0.f, b = 0.f;
        for (int l = 0; l < lanes; ++l) { a += red[0][l * G + gg][j]; b += red[1][l * G + gg][j]; }
        part[(size_t)blockIdx.x * 2 * C + c] = a;
        part[(size_t)blockIdx.x * 2 * C + C + c] = b;
    }
}

// dbeta = sum dz, dgamma = sum dz xh (fixed-order over the block partials); red2 = the same
// for the data-gradient pass
__global__ __launch_bounds__(64 * FIN_WAVES) void k_bn_bwd_finalize(int nblocks, int C, const float* __restrict__ part,
                                                                  float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                  float* __restrict__ red2, int accumulate) {
    __shared__ float red[2][FIN_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    float s = 0.f, q = 0.f;
    if (c < C) {
        for (int b = w; b < nblocks; b += FIN_WAVES) {
            s += part[(size_t)b * 2 * C + c];
            q += part[(size_t)b * 2 * C + C + c];
        }
    }
    red[0][w][lane] = s;
    red[1][w][lane] = q;
    __syncthreads();
    if (w != 0 || c >= C) return;
    s = 0.f;
    q = 0.f;
    for (int k = 0; k < FIN_WAVES; ++k) {
        s += red[0][k][lane];
        q += red[1][k][lane];
    }
    red2[c] = s;
    red2[C + c] = q;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + s : s;
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + q : q;
}

// dy = gamma rstd / N (N dz - sum dz - xh sum dz xh)
template <typename T>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(size_t nv, size_t npx, int C, const T* __restrict__ da,
                                                      const T* __restrict__ y, const float* __restrict__ stat,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float slope, const float* __restrict__ red2,
                                                      T* __restrict__ dy) {
    // (LDS-staged channel operands, as k_bn_apply, measured slower here: 13.0 -> 22.6 us)
    constexpr int V = 16 / sizeof(T);
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const int c0 = (int)((i * V) % C);
    float dv[V], yv[V];
    unpack16<T>(*(const uint4*)(da + i * V), dv);
    unpack16<T>(*(const uint4*)(y + i * V), yv);
    const float inv_n = 1.f / (float)npx;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = c0 + j;
        const float rs = stat[C + c];
        const float xh = (yv[j] - stat[c]) * rs;
        const float z = gamma[c] * xh + beta[c];
        const float dz = z > 0.f ? dv[j] : slope * dv[j];
        dv[j] = gamma[c] * rs * (dz - inv_n * red2[c] - xh * inv_n * red2[C + c]);
    }
    *(uint4*)(dy + i * V) = pack16<T>(dv);
}

// y[b][h][w] = x[b][2h][2w] (NHWC, 16 B per thread)
template <typename T>
__global__ __launch_bounds__(256) void k_subsample2(int B, int Ho, int Wo, int C, const T* __restrict__ x,
                                                    T* __restrict__ y) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * Ho * Wo * G) return;
    const int g = (int)(i % G);
    const size_t po = i / G;
    const int wo = (int)(po % Wo), ho = (int)((po / Wo) % Ho), b = (int)(po / ((size_t)Wo * Ho));
    const size_t src = (((size_t)b * 2 * Ho + 2 * ho) * (2 * Wo) + 2 * wo) * C + g * V;
    *(uint4*)(y + po * C + g * V) = *(const uint4*)(x + src);
}

// space-to-depth by 2 (the stride-2 conv's input as a stride-1 conv's, phase-major channels):
// s[b][i][j][(2a + c2) * C + c] = x[b][2i + a][2j + c2][c]; INV: x <- s (every element written)
template <typename T, bool INV>
__global__ __launch_bounds__(256) void k_s2d2(int B, int Ho, int Wo, int C, const T* __restrict__ src,
                                              T* __restrict__ dst) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // over s2d vectors
    if (i >= (size_t)B * Ho * Wo * 4 * G) return;
    const int g = (int)(i % G);
    const int ph = (int)((i / G) & 3);
    const size_t po = i / (4 * (size_t)G);
    const int wo = (int)(po % Wo), ho = (int)((po / Wo) % Ho), b = (int)(po / ((size_t)Wo * Ho));
    const size_t full = (((size_t)b * 2 * Ho + 2 * ho + (ph >> 1)) * (2 * Wo) + 2 * wo + (ph & 1)) * C + g * V;
    const size_t s2d = po * 4 * C + (size_t)ph * C + g * V;
    if constexpr (INV) *(uint4*)(dst + full) = *(const uint4*)(src + s2d);
    else *(uint4*)(dst + s2d) = *(const uint4*)(src + full);
}

// out[b][2h][2w] = dy[b][h][w], zero elsewhere (every element of out written)
template <typename T>
__global__ __launch_bounds__(256) void k_zero_insert2(int B, int Ho, int Wo, int C, const T* __restrict__ dy,
                                                      T* __restrict__ out) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;
    const int H = 2 * Ho, W = 2 * Wo;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * H * W * G) return;
    const int g = (int)(i % G);
    const size_t p = i / G;
    const int w = (int)(p % W), h = (int)((p / W) % H), b = (int)(p / ((size_t)W * H));
    uint4 v = make_uint4(0, 0, 0, 0);
    if (!(h & 1) && !(w & 1)) v = *(const uint4*)(dy + (((size_t)b * Ho + h / 2) * Wo + w / 2) * C + g * V);
    *(uint4*)(out + p * C + g * V) = v;
}

}  // namespace

#define STREAM ((hipStream_t)stream)
extern "C" size_t fen_bn_work_floats(int C) { return (size_t)BN_BLOCKS * 2 * C + 2 * C; }

// train-mode statistics of y (NHWC [npx][C]) -> stat [2C] (mean, rstd); running stats updated
// when rmean != NULL.  work: fen_bn_work_floats(C) floats.
extern "C" int fen_bn_stats(int dtype, size_t npx, int C, const void* y, float eps, float momentum, float* stat,
                            float* rmean, float* rvar, float* work, void* stream) {
    if (!y || !stat || !work || npx == 0 || C % 8 || C > 2048 || (rmean != nullptr) != (rvar != nullptr))
        return FEN_EINVAL;
    if (dtype == FEN_BF16) {
        hipLaunchKernelGGL(k_bn_stats<bf16>, dim3(BN_BLOCKS), dim3(256), 0, STREAM, npx, C, (const bf16*)y, work);
        FEN_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_bn_finalize<bf16>, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, STREAM, BN_BLOCKS, npx, C, (const bf16*)y,
                           work, eps, momentum, stat, rmean, rvar);
    } else if (dtype == FEN_F32) {
        hipLaunchKernelGGL(k_bn_stats<float>, dim3(BN_BLOCKS), dim3(256), 0, STREAM, npx, C, (const float*)y, work);
        FEN_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, STREAM, BN_BLOCKS, npx, C,
                           (const float*)y, work, eps, momentum, stat, rmean, rvar);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// out = lrelu((y - mean) * rstd * gamma + beta); mean / rstd = stat (train) or the running
// statistics turned into rstd by the caller (eval)
extern "C" int fen_bn_apply(int dtype, size_t npx, int C, const void* y, const float* mean, const float* rstd,
                            const float* gamma, const float* beta, float slope, void* out, void* stream) {
    if (!y || !mean || !rstd || !gamma || !beta || !out || C % 8) return FEN_EINVAL;
    if (C > 1024) return FEN_EUNSUPPORTED;
    if (dtype == FEN_BF16) {
        const size_t nv = npx * C / 8;
        hipLaunchKernelGGL(k_bn_apply<bf16>, dim3(nblk(nv, 256 * BN_NPT)), dim3(256), 0, STREAM, nv, C, (const bf16*)y,
                           mean, rstd, gamma, beta, slope, (bf16*)out);
    } else if (dtype == FEN_F32) {
        const size_t nv = npx * C / 4;
        hipLaunchKernelGGL(k_bn_apply<float>, dim3(nblk(nv, 256 * BN_NPT)), dim3(256), 0, STREAM, nv, C,
                           (const float*)y, mean, rstd, gamma, beta, slope, (float*)out);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// backward of out = lrelu(BN_train(y)): dy (NHWC) from da; dgamma / dbeta (accumulate or set)
extern "C" int fen_bn_bwd(int dtype, size_t npx, int C, const void* da, const void* y, const float* stat,
                          const float* gamma, const float* beta, float slope, void* dy, float* dgamma, float* dbeta,
                          int accumulate, float* work, void* stream) {
    if (!da || !y || !stat || !gamma || !beta || !dy || !work || C % 8 || C > 2048) return FEN_EINVAL;
    float* red2 = work + (size_t)BN_BLOCKS * 2 * C;
    if (dtype == FEN_BF16) {
        hipLaunchKernelGGL(k_bn_bwd_reduce<bf16>, dim3(BN_BLOCKS), dim3(256), 0, STREAM, npx, C, (const bf16*)da,
                           (const bf16*)y, stat, gamma, beta, slope, work);
    } else if (dtype == FEN_F32) {
        hipLaunchKernelGGL(k_bn_bwd_reduce<float>, dim3(BN_BLOCKS), dim3(256), 0, STREAM, npx, C, (const float*)da,
                           (const float*)y, stat, gamma, beta, slope, work);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, STREAM, BN_BLOCKS, C, work, dgamma, dbeta, red2,
                       accumulate);
    FEN_CHECK_LAUNCH();
    if (dtype == FEN_BF16) {
        const size_t nv = npx * C / 8;
        hipLaunchKernelGGL(k_bn_bwd_apply<bf16>, dim3(nblk(nv)), dim3(256), 0, STREAM, nv, npx, C, (const bf16*)da,
                           (const bf16*)y, stat, gamma, beta, slope, red2, (bf16*)dy);
    } else {
        const size_t nv = npx * C / 4;
        hipLaunchKernelGGL(k_bn_bwd_apply<float>, dim3(nblk(nv)), dim3(256), 0, STREAM, nv, npx, C, (const float*)da,
                           (const float*)y, stat, gamma, beta, slope, red2, (float*)dy);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_subsample2(int dtype, int B, int H, int W, int C, const void* x, void* y, void* stream) {
    if (!x || !y || (H | W) & 1 || C % 8) return FEN_EINVAL;
    if (dtype == FEN_BF16) {
        const size_t n = (size_t)B * (H / 2) * (W / 2) * (C / 8);
        hipLaunchKernelGGL(k_subsample2<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C, (const bf16*)x,
                           (bf16*)y);
    } else if (dtype == FEN_F32) {
        const size_t n = (size_t)B * (H / 2) * (W / 2) * (C / 4);
        hipLaunchKernelGGL(k_subsample2<float>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C,
                           (const float*)x, (float*)y);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_zero_insert2(int dtype, int B, int Ho, int Wo, int C, const void* dy, void* out, void* stream) {
    if (!dy || !out || C % 8) return FEN_EINVAL;
    if (dtype == FEN_BF16) {
        const size_t n = (size_t)B * 2 * Ho * 2 * Wo * (C / 8);
        hipLaunchKernelGGL(k_zero_insert2<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, Ho, Wo, C, (const bf16*)dy,
                           (bf16*)out);
    } else if (dtype == FEN_F32) {
        const size_t n = (size_t)B * 2 * Ho * 2 * Wo * (C / 4);
        hipLaunchKernelGGL(k_zero_insert2<float>, dim3(nblk(n)), dim3(256), 0, STREAM, B, Ho, Wo, C,
                           (const float*)dy, (float*)out);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_s2d2(int dtype, int B, int H, int W, int C, const void* x, void* y, int inverse, void* stream) {
    if (!x || !y || B <= 0 || H <= 0 || W <= 0 || (H | W) & 1 || C % 8) return FEN_EINVAL;
    const int V = dtype == FEN_F32 ? 4 : 8;
    const size_t n = (size_t)B * H * W * C / V;
    const int Ho = H / 2, Wo = W / 2;
    if (dtype == FEN_BF16 || dtype == FEN_F16) {
        if (inverse)
            hipLaunchKernelGGL((k_s2d2<bf16, true>), dim3(nblk(n)), dim3(256), 0, STREAM, B, Ho, Wo, C, (const bf16*)x,
                               (bf16*)y);
        else
            hipLaunchKernelGGL((k_s2d2<bf16, false>), dim3(nblk(n)), dim3(256), 0, STREAM, B, Ho, Wo, C, (const bf16*)x,
                               (bf16*)y);
    } else if (dtype == FEN_F32) {
        if (inverse)
            hipLaunchKernelGGL((k_s2d2<float, true>), dim3(nblk(n)), dim3(256), 0, STREAM, B, Ho, Wo, C, (const float*)x,
                               (float*)y);
        else
            hipLaunchKernelGGL((k_s2d2<float, false>), dim3(nblk(n)), dim3(256), 0, STREAM, B, Ho, Wo, C,
                               (const float*)x, (float*)y);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// The phase-major filter of a space-to-depth stride-2 conv (see fen_s2d2), fp32 OIHW:
// scatter: W' [Cout][4C][3][3] from W [Cout][C][3][3] (every element written, zeros where no
// tap of W lands); gather: dW [Cout][C][3][3] from dW'.  Tap kh -> (phase bit, kh'):
// 0 -> (1, 0), 1 -> (0, 1), 2 -> (1, 1); kw likewise.
template <bool GATHER>
__global__ __launch_bounds__(256) void k_s2d_filter(int Cout, int C, const float* __restrict__ src,
                                                    float* __restrict__ dst) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (GATHER) {
        if (i >= (size_t)Cout * C * 9) return;
        const int tap = (int)(i % 9), c = (int)((i / 9) % C), co = (int)(i / (9 * (size_t)C));
        const int kh = tap / 3, kw = tap % 3;
        const int a = kh == 1 ? 0 : 1, kh2 = kh == 0 ? 0 : 1;
        const int b = kw == 1 ? 0 : 1, kw2 = kw == 0 ? 0 : 1;
        dst[i] = src[((size_t)co * 4 * C + (2 * a + b) * C + c) * 9 + kh2 * 3 + kw2];
    } else {
        if (i >= (size_t)Cout * 4 * C * 9) return;
        const int tap = (int)(i % 9), cc = (int)((i / 9) % (4 * C)), co = (int)(i / (36 * (size_t)C));
        const int ph = cc / C, c = cc % C, a = ph >> 1, b = ph & 1;
        const int kh2 = tap / 3, kw2 = tap % 3;
        const bool live = kh2 <= 1 && kw2 <= 1 && (a || kh2 == 1) && (b || kw2 == 1);
        const int kh = a == 0 ? 1 : (kh2 == 0 ? 0 : 2), kw = b == 0 ? 1 : (kw2 == 0 ? 0 : 2);
        dst[i] = live ? src[((size_t)co * C + c) * 9 + kh * 3 + kw] : 0.f;
    }
}

extern "C" int fen_s2d_filter(int Cout, int C, const float* src, float* dst, int gather, void* stream) {
    if (!src || !dst || Cout <= 0 || C <= 0) return FEN_EINVAL;
    const size_t n = (size_t)Cout * C * 9 * (gather ? 1 : 4);
    if (gather) hipLaunchKernelGGL(k_s2d_filter<true>, dim3(nblk(n)), dim3(256), 0, STREAM, Cout, C, src, dst);
    else hipLaunchKernelGGL(k_s2d_filter<false>, dim3(nblk(n)), dim3(256), 0, STREAM, Cout, C, src, dst);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

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
// (blockIdx.y = group: groups of npx pixels one after another in y, partials [group][blk][2C])
template <typename T>
__global__ __launch_bounds__(256) void k_bn_stats(size_t npx, int C, const T* __restrict__ y,
                                                  float* __restrict__ part) {
    constexpr int V = 16 / sizeof(T);
    y += (size_t)blockIdx.y * npx * C;
    part += (size_t)blockIdx.y * gridDim.x * 2 * C;
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
// (one group per launch: a form walking the groups inside one launch measured 19-42 us per
// launch vs 6.2 per group -- the grouped entry points launch this once per group)
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
        // (unrolled: the partials' loads in flight together, summed in the same order -- the
        // rolled loop waited one L2 round trip per partial, ~12 us per finalize)
#pragma unroll 8
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
    da += (size_t)blockIdx.y * npx * C;                      // (blockIdx.y = group, as k_bn_stats)
    y += (size_t)blockIdx.y * npx * C;
    stat += (size_t)blockIdx.y * 2 * C;
    part += (size_t)blockIdx.y * gridDim.x * 2 * C;
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
#pragma unroll 8
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

// The same two elementwise passes with each thread on one fixed 16-B channel group (G = C / V
// groups, 256 / G pixel lanes, BN_PPT pixels per thread with their loads in flight): the group's
// per-channel operands are loaded into registers once per thread, not per vector (the forms
// above index them per vector with a 64-bit modulo).  Arithmetic unchanged: bit-identical.
constexpr int BN_PPT = 4;
// (blockIdx.y = group: y / out advance npx pixels, mean / rstd `mstride` floats per group)
template <typename T>
__global__ __launch_bounds__(256) void k_bn_apply_g(size_t npx, int C, const T* __restrict__ y,
                                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float slope, T* __restrict__ out, int mstride) {
    constexpr int V = 16 / sizeof(T);
    y += (size_t)blockIdx.y * npx * C;
    out += (size_t)blockIdx.y * npx * C;
    mean += (size_t)blockIdx.y * mstride;
    rstd += (size_t)blockIdx.y * mstride;
    const int G = C / V, lanes = 256 / G;
    const int g = threadIdx.x % G, pl = threadIdx.x / G;
    if (pl >= lanes) return;
    float sm[V], sr[V], sg[V], sb[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = g * V + j;
        sm[j] = mean[c], sr[j] = rstd[c], sg[j] = gamma[c], sb[j] = beta[c];
    }
    const size_t p0 = (size_t)blockIdx.x * lanes * BN_PPT + pl;
    uint4 d[BN_PPT];
#pragma unroll
    for (int k = 0; k < BN_PPT; ++k) {
        const size_t p = p0 + (size_t)k * lanes;
        if (p < npx) d[k] = *(const uint4*)(y + p * C + g * V);
    }
#pragma unroll
    for (int k = 0; k < BN_PPT; ++k) {
        const size_t p = p0 + (size_t)k * lanes;
        if (p >= npx) break;
        float v[V];
        unpack16<T>(d[k], v);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float z = (v[j] - sm[j]) * sr[j] * sg[j] + sb[j];
            v[j] = z > 0.f ? z : slope * z;
        }
        *(uint4*)(out + p * C + g * V) = pack16<T>(v);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_bn_bwd_apply_g(size_t npx, int C, const T* __restrict__ da,
                                                        const T* __restrict__ y, const float* __restrict__ stat,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        float slope, const float* __restrict__ red2,
                                                        T* __restrict__ dy) {
    constexpr int V = 16 / sizeof(T);
    da += (size_t)blockIdx.y * npx * C;                      // (blockIdx.y = group)
    y += (size_t)blockIdx.y * npx * C;
    dy += (size_t)blockIdx.y * npx * C;
    stat += (size_t)blockIdx.y * 2 * C;
    red2 += (size_t)blockIdx.y * 2 * C;
    const int G = C / V, lanes = 256 / G;
    const int g = threadIdx.x % G, pl = threadIdx.x / G;
    if (pl >= lanes) return;
    float mu[V], rs[V], ga[V], be[V], s0[V], s1[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = g * V + j;
        mu[j] = stat[c], rs[j] = stat[C + c], ga[j] = gamma[c], be[j] = beta[c], s0[j] = red2[c], s1[j] = red2[C + c];
    }
    const float inv_n = 1.f / (float)npx;
    const size_t p0 = (size_t)blockIdx.x * lanes * BN_PPT + pl;
    uint4 dd[BN_PPT], yy[BN_PPT];
#pragma unroll
    for (int k = 0; k < BN_PPT; ++k) {
        const size_t p = p0 + (size_t)k * lanes;
        if (p < npx) {
            dd[k] = *(const uint4*)(da + p * C + g * V);
            yy[k] = *(const uint4*)(y + p * C + g * V);
        }
    }
#pragma unroll
    for (int k = 0; k < BN_PPT; ++k) {
        const size_t p = p0 + (size_t)k * lanes;
        if (p >= npx) break;
        float dv[V], yv[V];
        unpack16<T>(dd[k], dv);
        unpack16<T>(yy[k], yv);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float xh = (yv[j] - mu[j]) * rs[j];
            const float z = ga[j] * xh + be[j];
            const float dz = z > 0.f ? dv[j] : slope * dv[j];
            dv[j] = ga[j] * rs[j] * (dz - inv_n * s0[j] - xh * inv_n * s1[j]);
        }
        *(uint4*)(dy + p * C + g * V) = pack16<T>(dv);
    }
}
}  // namespace

#define STREAM ((hipStream_t)stream)
extern "C" size_t fen_bn_work_floats(int C) { return (size_t)BN_BLOCKS * 2 * C + 2 * C; }

// train-mode statistics of ng groups of npx pixels each, one after another in y (NHWC) -> stat
// [ng][2C] (mean, rstd); running stats updated group by group in order when rmean != NULL.
// work: ng * fen_bn_work_floats(C) floats.  The statistics pass is one launch whatever ng (the D
// step's real and fake batches), the finalize one per group; bit-identical to per-group calls
extern "C" int fen_bn_stats_n(int dtype, int ng, size_t npx, int C, const void* y, float eps, float momentum,
                              float* stat, float* rmean, float* rvar, float* work, void* stream) {
    if (!y || !stat || !work || npx == 0 || ng < 1 || ng > 65535 || C % 8 || C > 2048 ||
        (rmean != nullptr) != (rvar != nullptr))
        return FEN_EINVAL;
    if (dtype == FEN_BF16) {
        hipLaunchKernelGGL(k_bn_stats<bf16>, dim3(BN_BLOCKS, ng), dim3(256), 0, STREAM, npx, C, (const bf16*)y, work);
        FEN_CHECK_LAUNCH();
        for (int gi = 0; gi < ng; ++gi)                      // in group order: the running statistics
            hipLaunchKernelGGL(k_bn_finalize<bf16>, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, STREAM, BN_BLOCKS, npx, C,
                               (const bf16*)y + (size_t)gi * npx * C, work + (size_t)gi * BN_BLOCKS * 2 * C, eps, momentum,
                               stat + (size_t)gi * 2 * C, rmean, rvar);
    } else if (dtype == FEN_F32) {
        hipLaunchKernelGGL(k_bn_stats<float>, dim3(BN_BLOCKS, ng), dim3(256), 0, STREAM, npx, C, (const float*)y, work);
        FEN_CHECK_LAUNCH();
        for (int gi = 0; gi < ng; ++gi)
            hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, STREAM, BN_BLOCKS, npx, C,
                               (const float*)y + (size_t)gi * npx * C, work + (size_t)gi * BN_BLOCKS * 2 * C, eps, momentum,
                               stat + (size_t)gi * 2 * C, rmean, rvar);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// one group: stat [2C], work fen_bn_work_floats(C)
extern "C" int fen_bn_stats(int dtype, size_t npx, int C, const void* y, float eps, float momentum, float* stat,
                            float* rmean, float* rvar, float* work, void* stream) {
    return fen_bn_stats_n(dtype, 1, npx, C, y, eps, momentum, stat, rmean, rvar, work, stream);
}

// out = lrelu((y - mean) * rstd * gamma + beta) for ng groups of npx pixels (y / out one group
// after another; group g's mean / rstd at mean / rstd + g * mstride); mean / rstd = stat (train)
// or the running statistics turned into rstd by the caller (eval)
extern "C" int fen_bn_apply_n(int dtype, int ng, size_t npx, int C, const void* y, const float* mean, const float* rstd,
                              int mstride, const float* gamma, const float* beta, float slope, void* out,
                              void* stream) {
    if (!y || !mean || !rstd || !gamma || !beta || !out || C % 8 || ng < 1 || ng > 65535 || (ng > 1 && mstride < C))
        return FEN_EINVAL;
    if (C > 1024) return FEN_EUNSUPPORTED;
    if (dtype != FEN_BF16 && dtype != FEN_F32) return FEN_EINVAL;
    const int G = C / (dtype == FEN_F32 ? 4 : 8);
    if (G <= 256 && 256 % G == 0) {
        const size_t per = (size_t)(256 / G) * BN_PPT;
        const unsigned nb = (unsigned)((npx + per - 1) / per);
        if (dtype == FEN_BF16)
            hipLaunchKernelGGL(k_bn_apply_g<bf16>, dim3(nb, ng), dim3(256), 0, STREAM, npx, C, (const bf16*)y, mean, rstd,
                               gamma, beta, slope, (bf16*)out, mstride);
        else
            hipLaunchKernelGGL(k_bn_apply_g<float>, dim3(nb, ng), dim3(256), 0, STREAM, npx, C, (const float*)y, mean,
                               rstd, gamma, beta, slope, (float*)out, mstride);
        FEN_CHECK_LAUNCH();
        return FEN_OK;
    }
    const size_t esz = dtype == FEN_F32 ? 4 : 2;
    for (int gi = 0; gi < ng; ++gi) {                        // other channel counts: a launch per group
        const char* yg = (const char*)y + (size_t)gi * npx * C * esz;
        char* og = (char*)out + (size_t)gi * npx * C * esz;
        const float *mg = mean + (size_t)gi * mstride, *rg = rstd + (size_t)gi * mstride;
        if (dtype == FEN_BF16) {
            const size_t nv = npx * C / 8;
            hipLaunchKernelGGL(k_bn_apply<bf16>, dim3(nblk(nv, 256 * BN_NPT)), dim3(256), 0, STREAM, nv, C, (const bf16*)yg,
                               mg, rg, gamma, beta, slope, (bf16*)og);
        } else {
            const size_t nv = npx * C / 4;
            hipLaunchKernelGGL(k_bn_apply<float>, dim3(nblk(nv, 256 * BN_NPT)), dim3(256), 0, STREAM, nv, C,
                               (const float*)yg, mg, rg, gamma, beta, slope, (float*)og);
        }
        FEN_CHECK_LAUNCH();
    }
    return FEN_OK;
}

extern "C" int fen_bn_apply(int dtype, size_t npx, int C, const void* y, const float* mean, const float* rstd,
                            const float* gamma, const float* beta, float slope, void* out, void* stream) {
    return fen_bn_apply_n(dtype, 1, npx, C, y, mean, rstd, 0, gamma, beta, slope, out, stream);
}

// backward of out = lrelu(BN_train(y)) for ng groups of npx pixels (da / y / dy one group after
// another, stat [ng][2C]): dy from da; dgamma / dbeta = the groups' sums in order (group 0 set or
// accumulated as `accumulate` says).  work: ng * fen_bn_work_floats(C) floats.  The reduce and
// apply passes one launch whatever ng, the finalize one per group; bit-identical to ng calls of fen_bn_bwd with accumulate = (g > 0 || accumulate)
extern "C" int fen_bn_bwd_n(int dtype, int ng, size_t npx, int C, const void* da, const void* y, const float* stat,
                            const float* gamma, const float* beta, float slope, void* dy, float* dgamma, float* dbeta,
                            int accumulate, float* work, void* stream) {
    if (!da || !y || !stat || !gamma || !beta || !dy || !work || C % 8 || C > 2048 || ng < 1 || ng > 65535)
        return FEN_EINVAL;
    if (dtype != FEN_BF16 && dtype != FEN_F32) return FEN_EINVAL;
    float* red2 = work + (size_t)ng * BN_BLOCKS * 2 * C;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_bn_bwd_reduce<bf16>, dim3(BN_BLOCKS, ng), dim3(256), 0, STREAM, npx, C, (const bf16*)da,
                           (const bf16*)y, stat, gamma, beta, slope, work);
    else
        hipLaunchKernelGGL(k_bn_bwd_reduce<float>, dim3(BN_BLOCKS, ng), dim3(256), 0, STREAM, npx, C, (const float*)da,
                           (const float*)y, stat, gamma, beta, slope, work);
    FEN_CHECK_LAUNCH();
    for (int gi = 0; gi < ng; ++gi)                          // in group order: dgamma / dbeta accumulate
        hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, STREAM, BN_BLOCKS, C,
                           work + (size_t)gi * BN_BLOCKS * 2 * C, dgamma, dbeta, red2 + (size_t)gi * 2 * C,
                           gi ? 1 : accumulate);
    FEN_CHECK_LAUNCH();
    const int G = C / (dtype == FEN_F32 ? 4 : 8);
    if (G <= 256 && 256 % G == 0) {
        const size_t per = (size_t)(256 / G) * BN_PPT;
        const unsigned nb = (unsigned)((npx + per - 1) / per);
        if (dtype == FEN_BF16)
            hipLaunchKernelGGL(k_bn_bwd_apply_g<bf16>, dim3(nb, ng), dim3(256), 0, STREAM, npx, C, (const bf16*)da,
                               (const bf16*)y, stat, gamma, beta, slope, red2, (bf16*)dy);
        else
            hipLaunchKernelGGL(k_bn_bwd_apply_g<float>, dim3(nb, ng), dim3(256), 0, STREAM, npx, C, (const float*)da,
                               (const float*)y, stat, gamma, beta, slope, red2, (float*)dy);
        FEN_CHECK_LAUNCH();
        return FEN_OK;
    }
    const size_t esz = dtype == FEN_F32 ? 4 : 2;
    for (int gi = 0; gi < ng; ++gi) {                        // other channel counts: a launch per group
        const size_t o = (size_t)gi * npx * C * esz;
        const float* sg = stat + (size_t)gi * 2 * C;
        const float* rg = red2 + (size_t)gi * 2 * C;
        if (dtype == FEN_BF16) {
            const size_t nv = npx * C / 8;
            hipLaunchKernelGGL(k_bn_bwd_apply<bf16>, dim3(nblk(nv)), dim3(256), 0, STREAM, nv, npx, C,
                               (const bf16*)((const char*)da + o), (const bf16*)((const char*)y + o), sg, gamma, beta, slope,
                               rg, (bf16*)((char*)dy + o));
        } else {
            const size_t nv = npx * C / 4;
            hipLaunchKernelGGL(k_bn_bwd_apply<float>, dim3(nblk(nv)), dim3(256), 0, STREAM, nv, npx, C,
                               (const float*)((const char*)da + o), (const float*)((const char*)y + o), sg, gamma, beta,
                               slope, rg, (float*)((char*)dy + o));
        }
        FEN_CHECK_LAUNCH();
    }
    return FEN_OK;
}

extern "C" int fen_bn_bwd(int dtype, size_t npx, int C, const void* da, const void* y, const float* stat,
                          const float* gamma, const float* beta, float slope, void* dy, float* dgamma, float* dbeta,
                          int accumulate, float* work, void* stream) {
    return fen_bn_bwd_n(dtype, 1, npx, C, da, y, stat, gamma, beta, slope, dy, dgamma, dbeta, accumulate, work, stream);
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

// ---------------------------------------------------------------------------------------------
// The classifier head (discriminator.py:85-90: Flatten -> Linear(K, N) -> LeakyReLU(0.2) ->
// Linear(N, 1), optional sigmoid 131-132), fp32 as the reference.  K = 512 x 8 x 8 = 32768,
// N = 1024: the first layer's 128-MB weight is the whole cost -- one read in the forward, one read
// (for d(x)) and one write (its gradient) in the backward; everything else is small.
//   forward   k_dhead_mm: per k-split s, part[s][b][n] = sum_k x[b][k] w1[n][k] on fp32 MFMAs
//             (v_mfma_f32_16x16x4f32, a wave = 16 rows n x 16 samples, the weight row read as
//             float4 along k); k_dhead_fin: pre = b1 + sum_s part (fixed order), the LeakyReLU, the
//             second layer's dot (fixed-order block reduction), + b2 (and the sigmoid).
//   backward  k_dhead_bvec: dpre = g w2 LeakyReLU'(pre), db1, dw2, db2; k_dhead_bw: one wave per
//             256 k x N/G rows -- dw1[n][k] = sum_b dpre[b][n] x[b][k] (written once) and the
//             d(x) partial sum_n dpre[b][n] w1[n][k] over its rows (w1 read once), G row groups
//             summed by k_dhead_dxfin in fixed order.  Deterministic run to run.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int DH_SPLIT = 32;    // k-splits of the forward GEMM
constexpr int DH_G = 8;         // row groups of the backward's d(x)
constexpr int DH_BC = 16;       // samples per pass of the backward kernel
constexpr int DH_UNR = 8;       // forward: k-steps of loads in flight per wave
constexpr int DH_RUN = 4;       // backward: rows of loads in flight per wave

// the head's weight and its gradient are streamed once per launch: non-temporal (no L2 / MALL
// allocation for 128 MB that will not be re-read before it is evicted)
__device__ __forceinline__ float4 ld_nt4(const float* p) {
    const f32x4 v = __builtin_nontemporal_load((const f32x4*)p);
    return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_nt4(float* p, const float4& v) {
    __builtin_nontemporal_store((f32x4){v.x, v.y, v.z, v.w}, (f32x4*)p);
}

// NBB sample blocks of 16 per pass (bb0 .. bb0 + NBB - 1), their accumulators side by side: the
// weight rows stream from HBM once per pass -- once per launch for B <= 16 * DH_MAXBB (the D
// step's real + fake batches: 32 samples; one pass per 16 samples read the 128-MB weight twice)
constexpr int DH_MAXBB = 2;
template <int NBB>
__global__ __launch_bounds__(256) void k_dhead_mm(int B, int K, int N, int kc, int bb0, const float* __restrict__ x,
                                                  const float* __restrict__ w1, float* __restrict__ part) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int n0 = (blockIdx.x * 4 + wave) * 16;
    const int s = blockIdx.y;
    const int k0 = s * kc;
    const float* wrow = w1 + (size_t)(n0 + r) * K + k0 + 4 * q;
    const float* xrow[NBB];
    float xm[NBB];
    f32x4 acc[NBB];
#pragma unroll
    for (int i = 0; i < NBB; ++i) {
        const int b = (bb0 + i) * 16 + r;
        xrow[i] = x + (size_t)(b < B ? b : 0) * K + k0 + 4 * q;
        xm[i] = b < B ? 1.f : 0.f;
        acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // DH_UNR k-steps of loads in flight per wave
    for (int k = 0; k < kc; k += 16 * DH_UNR) {
        float4 wv[DH_UNR], xv[NBB][DH_UNR];
#pragma unroll
        for (int u = 0; u < DH_UNR; ++u) {
            wv[u] = ld_nt4(wrow + k + 16 * u);
#pragma unroll
            for (int i = 0; i < NBB; ++i) xv[i][u] = *(const float4*)(xrow[i] + k + 16 * u);
        }
#pragma unroll
        for (int u = 0; u < DH_UNR; ++u)
#pragma unroll
            for (int i = 0; i < NBB; ++i) {
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u].x, xv[i][u].x * xm[i], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u].y, xv[i][u].y * xm[i], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u].z, xv[i][u].z * xm[i], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u].w, xv[i][u].w * xm[i], acc[i], 0, 0, 0);
            }
    }
    // lane holds D[n0 + 4q + t][b] for t = 0..3
#pragma unroll
    for (int i = 0; i < NBB; ++i) {
        const int b = (bb0 + i) * 16 + r;
        if (b < B)
            *(float4*)(part + ((size_t)s * B + b) * N + n0 + 4 * q) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
    }
}

// one block per sample, one thread per output unit n (N <= 1024): the DH_SPLIT partials in
// fixed order (all loads in flight), the LeakyReLU, the second layer's dot by a fixed-order tree
__global__ __launch_bounds__(1024) void k_dhead_fin(int B, int N, int S, const float* __restrict__ part,
                                                    const float* __restrict__ b1, const float* __restrict__ w2,
                                                    const float* __restrict__ b2, float slope, int sigmoid,
                                                    float* __restrict__ pre, float* __restrict__ y) {
    __shared__ float red[1024];
    const int b = blockIdx.x, n = threadIdx.x;
    float acc = 0.f;
    if (n < N) {
        float pv[DH_SPLIT];
#pragma unroll
        for (int s = 0; s < DH_SPLIT; ++s) pv[s] = s < S ? part[((size_t)s * B + b) * N + n] : 0.f;
        float v = b1[n];
#pragma unroll
        for (int s = 0; s < DH_SPLIT; ++s)
            if (s < S) v += pv[s];
        pre[(size_t)b * N + n] = v;
        acc = (v > 0.f ? v : slope * v) * w2[n];
    }
    red[n] = acc;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (n < o) red[n] += red[n + o];
        __syncthreads();
    }
    if (n == 0) {
        const float sc = red[0] + b2[0];
        y[b] = sigmoid ? 1.f / (1.f + expf(-sc)) : sc;
    }
}

__global__ __launch_bounds__(256) void k_dhead_bvec(int B, int N, const float* __restrict__ gy,
                                                    const float* __restrict__ pre, const float* __restrict__ w2,
                                                    const float* __restrict__ y, float slope, int sigmoid,
                                                    float* __restrict__ dpre, float* __restrict__ db1,
                                                    float* __restrict__ dw2, float* __restrict__ db2) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n < N) {
        const float w = w2[n];
        float sdb = 0.f, sdw = 0.f;
        for (int b = 0; b < B; ++b) {
            const float g = sigmoid ? gy[b] * y[b] * (1.f - y[b]) : gy[b];
            const float p = pre[(size_t)b * N + n];
            const float dp = g * w * (p > 0.f ? 1.f : slope);
            dpre[(size_t)n * B + b] = dp;                     // [n][b]: the backward kernel's rows
            sdb += dp;
            sdw = fmaf(g, p > 0.f ? p : slope * p, sdw);
        }
        db1[n] = sdb;
        dw2[n] = sdw;
    }
    if (n == 0) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += sigmoid ? gy[b] * y[b] * (1.f - y[b]) : gy[b];
        db2[0] = s;
    }
}

// block = 4 waves over one 256-k column block and one group of N / DH_G rows (the waves take every
// 4th row): dw1[n][k] = sum_b dpre[n][b] x[b][k] written once, each wave's d(x) partial over its
// rows summed across the waves in LDS (fixed order) into dxpart[g]; dpre of the rows staged in
// LDS (read as broadcast float4s); samples [b0, b0 + nb) of this pass (accumulate: dw1 +=)
__global__ __launch_bounds__(256) void k_dhead_bw(int B, int K, int N, int b0, int nb, const float* __restrict__ x,
                                                  const float* __restrict__ w1, const float* __restrict__ dpre,
                                                  int accumulate, float* __restrict__ dw1, float* __restrict__ dxpart) {
    __shared__ __attribute__((aligned(16))) float sdp[1024 / DH_G * DH_BC];   // [row][b]
    __shared__ __attribute__((aligned(16))) float4 sdx[3][DH_BC][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int k4 = blockIdx.x * 256 + lane * 4;
    const int g = blockIdx.y;
    const int rows = N / DH_G, n0 = g * rows;
    for (int i = threadIdx.x; i < rows * DH_BC; i += 256) {
        const int rr = i / DH_BC, b = i % DH_BC;
        sdp[i] = b < nb ? dpre[(size_t)(n0 + rr) * B + b0 + b] : 0.f;
    }
    float4 xv[DH_BC], dx[DH_BC];
#pragma unroll
    for (int b = 0; b < DH_BC; ++b) {
        xv[b] = b < nb ? *(const float4*)(x + (size_t)(b0 + b) * K + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        dx[b] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    for (int rr = wave; rr < rows; rr += 4 * DH_RUN) {
        float4 wv[DH_RUN], dw[DH_RUN];
#pragma unroll
        for (int u = 0; u < DH_RUN; ++u) {
            const int n = n0 + rr + 4 * u;
            wv[u] = ld_nt4(w1 + (size_t)n * K + k4);
            dw[u] = accumulate ? *(const float4*)(dw1 + (size_t)n * K + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < DH_RUN; ++u) {
            const float4* dp4 = (const float4*)(sdp + (rr + 4 * u) * DH_BC);
#pragma unroll
            for (int b4 = 0; b4 < DH_BC / 4; ++b4) {
                const float4 p = dp4[b4];
                const float pb[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int b = 4 * b4 + j;
                    const float dp = pb[j];
                    dx[b].x = fmaf(dp, wv[u].x, dx[b].x), dx[b].y = fmaf(dp, wv[u].y, dx[b].y);
                    dx[b].z = fmaf(dp, wv[u].z, dx[b].z), dx[b].w = fmaf(dp, wv[u].w, dx[b].w);
                    dw[u].x = fmaf(dp, xv[b].x, dw[u].x), dw[u].y = fmaf(dp, xv[b].y, dw[u].y);
                    dw[u].z = fmaf(dp, xv[b].z, dw[u].z), dw[u].w = fmaf(dp, xv[b].w, dw[u].w);
                }
            }
            st_nt4(dw1 + (size_t)(n0 + rr + 4 * u) * K + k4, dw[u]);
        }
    }
    if (!dxpart) return;
    // the 4 waves' partials, summed in wave order
    if (wave > 0) {
#pragma unroll
        for (int b = 0; b < DH_BC; ++b) sdx[wave - 1][b][lane] = dx[b];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int b = 0; b < DH_BC; ++b) {
            if (b >= nb) continue;
            float4 v = dx[b];
#pragma unroll
            for (int w = 0; w < 3; ++w) {
                const float4 o = sdx[w][b][lane];
                v.x += o.x, v.y += o.y, v.z += o.z, v.w += o.w;
            }
            *(float4*)(dxpart + ((size_t)g * B + b0 + b) * K + k4) = v;
        }
    }
}

__global__ __launch_bounds__(256) void k_dhead_dxfin(size_t n, const float* __restrict__ dxpart, float* __restrict__ dx) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < DH_G; ++g) v += dxpart[(size_t)g * n + i];
    dx[i] = v;
}
// GANLoss (discriminator.py:154-206) against a constant label t, mean over n scores, one block
// (fixed-order reduction: deterministic):
//   mode 0 'vanilla': nn.BCEWithLogitsLoss, torch's stable form (1 - t) x + m + log(exp(-m) +
//                     exp(-x - m)), m = max(-x, 0); d/dx = sigmoid(x) - t
//   mode 1 'lsgan':   nn.MSELoss, (x - t)^2; d/dx = 2 (x - t)
//   mode 2 'wgan':    t x (t = -1 real, +1 fake: -mean / +mean); d/dx = t
// and the gradient gx = d/dx / n * gy, the upstream gradient gy read on the device.  n is the
// batch (16-32 scores): one launch each way instead of the ~10 small aten kernels per call.
__device__ __forceinline__ float gan_term(int mode, float v, float t) {
    if (mode == 0) {
        const float m = fmaxf(-v, 0.f);
        return (1.f - t) * v + m + logf(expf(-m) + expf(-v - m));
    }
    if (mode == 1) return (v - t) * (v - t);
    return t * v;
}

__global__ __launch_bounds__(256) void k_gan_loss(int mode, int n, const float* __restrict__ x, float t,
                                                   float* __restrict__ loss) {
    __shared__ float red[256];
    float a = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) a += gan_term(mode, x[i], t);
    red[threadIdx.x] = a;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = red[0] / (float)n;
}

__global__ __launch_bounds__(256) void k_gan_loss_bwd(int mode, int n, const float* __restrict__ x, float t,
                                                       const float* __restrict__ gy, float* __restrict__ gx) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    const float d = mode == 0 ? 1.f / (1.f + expf(-v)) - t : mode == 1 ? 2.f * (v - t) : t;
    gx[i] = d / (float)n * gy[0];
}

}  // namespace

extern "C" size_t fen_dhead_work_floats(int B, int K, int N) {
    if (B <= 0 || K <= 0 || N <= 0) return 0;
    const size_t fwd = (size_t)DH_SPLIT * B * N;
    const size_t bwd = (size_t)B * N + (size_t)DH_G * B * K;
    return fwd > bwd ? fwd : bwd;
}

// k-splits of the forward: the largest power of two <= DH_SPLIT whose chunks are whole unrolled steps
static int dhead_split(int K) {
    int S = DH_SPLIT;
    while (S > 1 && K % (16 * DH_UNR * S)) S >>= 1;
    return S;
}
static bool dhead_shape_ok(int B, int K, int N) {
    return B > 0 && K % (16 * DH_UNR) == 0 && K % 256 == 0 && N % 64 == 0 && N <= 1024 && (N / DH_G) % (4 * DH_RUN) == 0;
}

extern "C" int fen_dhead_fwd(int B, int K, int N, const float* x, const float* w1, const float* b1, const float* w2,
                             const float* b2, float slope, int sigmoid, float* pre, float* y, float* work,
                             void* stream) {
    if (!x || !w1 || !b1 || !w2 || !b2 || !pre || !y || !work || B <= 0 || K <= 0 || N <= 0) return FEN_EINVAL;
    if (!dhead_shape_ok(B, K, N)) return FEN_EUNSUPPORTED;
    const int S = dhead_split(K), kc = K / S;
    const int nbb = (B + 15) >> 4;
    for (int bb = 0; bb < nbb; bb += DH_MAXBB) {             // one pass for B <= 32
        if (nbb - bb >= 2)
            hipLaunchKernelGGL(k_dhead_mm<2>, dim3(N / 64, S), dim3(256), 0, STREAM, B, K, N, kc, bb, x, w1, work);
        else
            hipLaunchKernelGGL(k_dhead_mm<1>, dim3(N / 64, S), dim3(256), 0, STREAM, B, K, N, kc, bb, x, w1, work);
    }
    hipLaunchKernelGGL(k_dhead_fin, dim3(B), dim3(1024), 0, STREAM, B, N, S, work, b1, w2, b2, slope, sigmoid, pre, y);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_dhead_bwd(int B, int K, int N, const float* x, const float* w1, const float* pre, const float* w2,
                             const float* y, const float* gy, float slope, int sigmoid, float* dx, float* dw1,
                             float* db1, float* dw2, float* db2, float* work, void* stream) {
    if (!x || !w1 || !pre || !w2 || !gy || !dw1 || !db1 || !dw2 || !db2 || !work || (sigmoid && !y)) return FEN_EINVAL;
    if (!dhead_shape_ok(B, K, N)) return FEN_EUNSUPPORTED;
    float* dpre = work;
    float* dxpart = dx ? work + (size_t)B * N : nullptr;
    hipLaunchKernelGGL(k_dhead_bvec, dim3((N + 255) / 256), dim3(256), 0, STREAM, B, N, gy, pre, w2, y, slope, sigmoid,
                       dpre, db1, dw2, db2);
    for (int b0 = 0; b0 < B; b0 += DH_BC) {
        const int nb = B - b0 < DH_BC ? B - b0 : DH_BC;
        hipLaunchKernelGGL(k_dhead_bw, dim3(K / 256, DH_G), dim3(256), 0, STREAM, B, K, N, b0, nb, x, w1, dpre,
                           b0 > 0 ? 1 : 0, dw1, dxpart);
    }
    if (dx) {
        const size_t n = (size_t)B * K;
        hipLaunchKernelGGL(k_dhead_dxfin, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, STREAM, n, dxpart, dx);
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_gan_loss(int mode, int n, const float* x, float target, float* loss, void* stream) {
    if (mode < 0 || mode > 2 || n <= 0 || !x || !loss) return FEN_EINVAL;
    hipLaunchKernelGGL(k_gan_loss, dim3(1), dim3(256), 0, STREAM, mode, n, x, target, loss);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_gan_loss_bwd(int mode, int n, const float* x, float target, const float* gy, float* gx,
                                void* stream) {
    if (mode < 0 || mode > 2 || n <= 0 || !x || !gy || !gx) return FEN_EINVAL;
    hipLaunchKernelGGL(k_gan_loss_bwd, dim3((n + 255) / 256), dim3(256), 0, STREAM, mode, n, x, target, gy, gx);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

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

namespace {

constexpr int SR = 5;       // window radius (window 11)
constexpr int ST = 32;      // output tile
struct SsimWin {
    float g[2 * SR + 1];
};

inline int nblk(size_t n, int t = 256) { return (int)((n + t - 1) / t); }

template <bool GRAD, typename T>
__global__ __launch_bounds__(256) void k_ssim(int B, int C, int H, int W, const float* __restrict__ pred,
                                              const float* __restrict__ target, const SsimWin win, float C1,
                                              float C2, float* __restrict__ part, void* __restrict__ grad,
                                              float grad_scale, int grad_mode) {
    constexpr int E1 = GRAD ? ST + 2 * SR : ST;   // where the map (and a, b, c) is needed
    constexpr int E2 = E1 + 2 * SR;               // where the inputs are needed
    constexpr int O1 = GRAD ? SR : 0;             // tile offset inside E1
    __shared__ float sp[E2][E2 + 1], st[E2][E2 + 1];
    __shared__ float hp[5][E2][E1 + 1];           // horizontal pass (reused for a, b, c)
    __shared__ float abc[3][E1][E1 + 1];
    __shared__ float red[256];
    const int tid = threadIdx.x;
    const int plane = blockIdx.z, b = plane / C, ch = plane % C;
    const int h0 = blockIdx.y * ST, w0 = blockIdx.x * ST;
    const int gy0 = h0 - O1 - SR, gx0 = w0 - O1 - SR;     // image coords of E2's (0, 0)
    const float* pp = pred + (size_t)plane * H * W;
    const float* tp = target + (size_t)plane * H * W;
    for (int i = tid; i < E2 * E2; i += 256) {
        const int r = i / E2, c = i % E2, gy = gy0 + r, gx = gx0 + c;
        const bool in = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
        sp[r][c] = in ? pp[(size_t)gy * W + gx] : 0.f;
        st[r][c] = in ? tp[(size_t)gy * W + gx] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < E2 * E1; i += 256) {
        const int r = i / E1, c = i % E1;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
        for (int j = 0; j < 2 * SR + 1; ++j) {
            const float p = sp[r][c + j], t = st[r][c + j], g = win.g[j];
            s0 += g * p; s1 += g * t; s2 += g * p * p; s3 += g * t * t; s4 += g * p * t;
        }
        hp[0][r][c] = s0; hp[1][r][c] = s1; hp[2][r][c] = s2; hp[3][r][c] = s3; hp[4][r][c] = s4;
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = tid; i < E1 * E1; i += 256) {
        const int r = i / E1, c = i % E1;
        float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2 * SR + 1; ++j) {
            const float g = win.g[j];
#pragma unroll
            for (int k = 0; k < 5; ++k) m[k] += g * hp[k][r + j][c];
        }
        const float mp = m[0], mt = m[1];
        const float spp = m[2] - mp * mp, stt = m[3] - mt * mt, spt = m[4] - mp * mt;
        const float A1 = 2.f * mp * mt + C1, A2 = 2.f * spt + C2;
        const float B1 = mp * mp + mt * mt + C1, B2 = spp + stt + C2;
        const float S = (A1 * A2) / (B1 * B2);
        const int gy = h0 - O1 + r, gx = w0 - O1 + c;
        const bool in = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
        const bool own = r >= O1 && r < O1 + ST && c >= O1 && c < O1 + ST;
        if (in && own) acc += S;
        if constexpr (GRAD) {
            const float iB = 1.f / (B1 * B2);
            abc[0][r][c] = in ? 2.f * mt * (A2 - A1) * iB - 2.f * mp * S * (1.f / B1 - 1.f / B2) : 0.f;
            abc[1][r][c] = in ? -S / B2 : 0.f;
            abc[2][r][c] = in ? 2.f * A1 * iB : 0.f;
        }
    }
    if constexpr (GRAD) {
        __syncthreads();
        for (int i = tid; i < E1 * ST; i += 256) {           // horizontal pass of a, b, c
            const int r = i / ST, c = i % ST;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int j = 0; j < 2 * SR + 1; ++j) {
                const float g = win.g[j];
                s0 += g * abc[0][r][c + j]; s1 += g * abc[1][r][c + j]; s2 += g * abc[2][r][c + j];
            }
            hp[0][r][c] = s0; hp[1][r][c] = s1; hp[2][r][c] = s2;
        }
        __syncthreads();
        for (int i = tid; i < ST * ST; i += 256) {
            const int r = i / ST, c = i % ST, gy = h0 + r, gx = w0 + c;
            if (gy >= H || gx >= W) continue;
            float ga = 0.f, gb = 0.f, gc = 0.f;
#pragma unroll
            for (int j = 0; j < 2 * SR + 1; ++j) {
                const float g = win.g[j];
                ga += g * hp[0][r + j][c]; gb += g * hp[1][r + j][c]; gc += g * hp[2][r + j][c];
            }
            const float p = sp[r + 2 * SR][c + 2 * SR], t = st[r + 2 * SR][c + 2 * SR];
            const float d = grad_scale * (ga + 2.f * p * gb + t * gc);
            if (grad_mode == 1) {
                ((float*)grad)[(size_t)plane * H * W + (size_t)gy * W + gx] = d;
            } else {
                T* o = (T*)grad + (((size_t)b * H + gy) * W + gx) * 16 + ch;
                *o = fromf<T>(tof<T>(*o) + d);
            }
        }
    }
    red[tid] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    if (tid == 0) {
        const int ntile = gridDim.x * gridDim.y;
        part[((size_t)ch * ntile + blockIdx.y * gridDim.x + blockIdx.x) * B + b] = red[0];
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
    if (grad_mode == 0) {
        hipLaunchKernelGGL((k_ssim<false, float>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, nullptr, 0.f, 0);
    } else if (grad_mode == 1 || dtype == FEN_F32) {
        hipLaunchKernelGGL((k_ssim<true, float>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode);
    } else if (dtype == FEN_BF16) {
        hipLaunchKernelGGL((k_ssim<true, bf16>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

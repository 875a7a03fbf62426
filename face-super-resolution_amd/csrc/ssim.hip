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

// Horizontal pass over NCH column chunks of CW outputs: thread keeps the CW + 10 inputs of
// its chunk in registers and reads each LDS element once.
template <int CW>
__device__ __forceinline__ void hrow(const SsimWin& win, const float* p, const float* t, float (&o)[5][CW]) {
    float pv[CW + 2 * SR], tv[CW + 2 * SR];
#pragma unroll
    for (int i = 0; i < CW + 2 * SR; ++i) { pv[i] = p[i]; tv[i] = t[i]; }
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
        for (int j = 0; j < 2 * SR + 1; ++j) {
            const float pp = pv[c + j], tt = tv[c + j], g = win.g[j];
            s0 += g * pp; s1 += g * tt; s2 += g * pp * pp; s3 += g * tt * tt; s4 += g * pp * tt;
        }
        o[0][c] = s0; o[1][c] = s1; o[2][c] = s2; o[3][c] = s3; o[4][c] = s4;
    }
}

// CB > 1 (grad_mode 2, C <= CB): one block takes every channel of its tile in turn and adds the
// gradients to the NHWC16 buffer once, 4 channels per 8-B (16-bit) / 16-B (fp32) read-modify-
// write per pixel, instead of C blocks each rewriting one 2-byte channel of every pixel row.
template <bool GRAD, typename T, int CB>
__global__ __launch_bounds__(256) void k_ssim(int B, int C, int H, int W, const float* __restrict__ pred,
                                              const float* __restrict__ target, const SsimWin win, float C1,
                                              float C2, float* __restrict__ part, void* __restrict__ grad,
                                              float grad_scale, int grad_mode) {
    constexpr int E1 = GRAD ? ST + 2 * SR : ST;   // where the map (and a, b, c) is needed
    constexpr int E2 = E1 + 2 * SR;               // where the inputs are needed
    constexpr int O1 = GRAD ? SR : 0;             // tile offset inside E1
    constexpr int CW = GRAD ? 7 : 8;              // register block of the map passes (E1 = 6 or 4 of them)
    constexpr int NCH = E1 / CW;
    constexpr int CW2 = 8, NCH2 = ST / CW2;       // register block of the gradient passes
    constexpr int PS = E2 + 1;
    // sb: p, t on E2 x E2; after the first pass, a / b / c on E1 x E1 (3 E1 (E1+1) <= 2 E2 PS)
    __shared__ float sb[2 * E2 * PS];
    __shared__ float hp[5][E2][E1 + 1];           // horizontal sums (reused for a, b, c)
    __shared__ float red[256];
    static_assert(3 * E1 * (E1 + 1) <= 2 * E2 * PS, "a/b/c alias");
    float* sp = sb;
    float* st = sb + E2 * PS;
    float (*abc)[E1][E1 + 1] = (float (*)[E1][E1 + 1])sb;
    const int tid = threadIdx.x;
    const int h0 = blockIdx.y * ST, w0 = blockIdx.x * ST;
    const int gy0 = h0 - O1 - SR, gx0 = w0 - O1 - SR;     // image coords of E2's (0, 0)
    const int b = CB > 1 ? (int)blockIdx.z : (int)blockIdx.z / C;
    float dacc[CB][CW2];                                  // CB > 1: this thread's gradients, per channel
#pragma unroll
    for (int k = 0; k < CB; ++k)
#pragma unroll
        for (int o = 0; o < CW2; ++o) dacc[k][o] = 0.f;
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
    for (int i = tid; i < E2 * NCH; i += 256) {
        const int r = i / NCH, c0 = (i % NCH) * CW;
        float o[5][CW];
        hrow<CW>(win, sp + r * PS + c0, st + r * PS + c0, o);
#pragma unroll
        for (int k = 0; k < 5; ++k)
#pragma unroll
            for (int c = 0; c < CW; ++c) hp[k][r][c0 + c] = o[k][c];
    }
    __syncthreads();
    // vertical pass: thread = (column, CW-row chunk), the chunk's CW + 10 rows read once
    float acc = 0.f;
    for (int i = tid; i < E1 * NCH; i += 256) {
        const int c = i % E1, r0 = (i / E1) * CW;
        float m[5][CW];
#pragma unroll
        for (int k = 0; k < 5; ++k)
#pragma unroll
            for (int o = 0; o < CW; ++o) m[k][o] = 0.f;
#pragma unroll
        for (int rr = 0; rr < CW + 2 * SR; ++rr) {
            float v[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) v[k] = hp[k][r0 + rr][c];
#pragma unroll
            for (int o = 0; o < CW; ++o) {
                const int j = rr - o;
                if (j >= 0 && j <= 2 * SR) {
#pragma unroll
                    for (int k = 0; k < 5; ++k) m[k][o] += win.g[j] * v[k];
                }
            }
        }
#pragma unroll
        for (int o = 0; o < CW; ++o) {
            const int r = r0 + o;
            const float mp = m[0][o], mt = m[1][o];
            const float spp = m[2][o] - mp * mp, stt = m[3][o] - mt * mt, spt = m[4][o] - mp * mt;
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
    }
    if constexpr (GRAD) {
        __syncthreads();
        for (int i = tid; i < E1 * NCH2; i += 256) {          // horizontal pass of a, b, c
            const int r = i / NCH2, c0 = (i % NCH2) * CW2;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                float v[CW2 + 2 * SR];
#pragma unroll
                for (int q = 0; q < CW2 + 2 * SR; ++q) v[q] = abc[k][r][c0 + q];
#pragma unroll
                for (int c = 0; c < CW2; ++c) {
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < 2 * SR + 1; ++j) s += win.g[j] * v[c + j];
                    hp[k][r][c0 + c] = s;
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < ST * NCH2; i += 256) {          // vertical pass + the gradient
            const int c = i % ST, r0 = (i / ST) * CW2, gx = w0 + c;
            float m[3][CW2];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int o = 0; o < CW2; ++o) m[k][o] = 0.f;
#pragma unroll
            for (int rr = 0; rr < CW2 + 2 * SR; ++rr) {
                float v[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) v[k] = hp[k][r0 + rr][c];
#pragma unroll
                for (int o = 0; o < CW2; ++o) {
                    const int j = rr - o;
                    if (j >= 0 && j <= 2 * SR) {
#pragma unroll
                        for (int k = 0; k < 3; ++k) m[k][o] += win.g[j] * v[k];
                    }
                }
            }
            if (gx >= W) continue;
            float pr[CW2], tr[CW2];                               // L2-hot: this block staged them
#pragma unroll
            for (int o = 0; o < CW2; ++o) {
                const int gy = min(h0 + r0 + o, H - 1);
                pr[o] = pp[(size_t)gy * W + gx];
                tr[o] = tp[(size_t)gy * W + gx];
            }
#pragma unroll
            for (int o = 0; o < CW2; ++o) {
                const int gy = h0 + r0 + o;
                if (gy >= H) break;
                const size_t e = (size_t)gy * W + gx;
                const float p = pr[o], t = tr[o];
                const float d = grad_scale * (m[0][o] + 2.f * p * m[1][o] + t * m[2][o]);
                if constexpr (CB > 1) {
                    dacc[cc][o] = d;
                } else if (grad_mode == 1) {
                    ((float*)grad)[(size_t)plane * H * W + e] = d;
                } else {
                    T* q = (T*)grad + (((size_t)b * H + gy) * W + gx) * 16 + ch;
                    *q = fromf<T>(tof<T>(*q) + d);
                }
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
    }   // channels
    if constexpr (GRAD && CB > 1) {
        // channels 0..3 of each pixel in one read-modify-write (channels >= C written back as read)
        for (int i = tid; i < ST * NCH2; i += 256) {
            const int c = i % ST, r0 = (i / ST) * CW2, gx = w0 + c;
            if (gx >= W) continue;
#pragma unroll
            for (int o = 0; o < CW2; ++o) {
                const int gy = h0 + r0 + o;
                if (gy >= H) break;
                T* q = (T*)grad + (((size_t)b * H + gy) * W + gx) * 16;
                if constexpr (sizeof(T) == 2) {
                    uint2 u = *(const uint2*)q;
                    const T* v = (const T*)&u;
                    T w4[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
                    for (int k = 0; k < CB && k < 4; ++k)
                        if (k < C) w4[k] = fromf<T>(tof<T>(w4[k]) + dacc[k][o]);
                    *(uint2*)q = *(const uint2*)w4;
                } else {
                    float4 u = *(const float4*)q;
                    float* v = (float*)&u;
#pragma unroll
                    for (int k = 0; k < CB && k < 4; ++k)
                        if (k < C) v[k] += dacc[k][o];
                    *(float4*)q = u;
                }
            }
        }
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
    if (grad_mode == 0) {
        hipLaunchKernelGGL((k_ssim<false, float, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, nullptr, 0.f, 0);
    } else if (grad_mode == 1) {
        hipLaunchKernelGGL((k_ssim<true, float, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode);
    } else if (C <= 3 && (dtype == FEN_F32 || dtype == FEN_BF16)) {
        if (dtype == FEN_F32)
            hipLaunchKernelGGL((k_ssim<true, float, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                               C2, part, grad, grad_scale, grad_mode);
        else
            hipLaunchKernelGGL((k_ssim<true, bf16, 3>), gridb, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1,
                               C2, part, grad, grad_scale, grad_mode);
    } else if (dtype == FEN_F32) {
        hipLaunchKernelGGL((k_ssim<true, float, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode);
    } else if (dtype == FEN_BF16) {
        hipLaunchKernelGGL((k_ssim<true, bf16, 1>), grid, dim3(256), 0, STREAM, B, C, H, W, pred, target, w, C1, C2,
                           part, grad, grad_scale, grad_mode);
    } else {
        return FEN_EINVAL;
    }
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

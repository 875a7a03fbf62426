// VGG19 perceptual-loss pieces (reference src/losses/perceptual.py:13-169) that the conv
// kernels do not already cover: the 2x2 max pool (torchvision vgg19.features 'M' layers,
// perceptual.py:50-53) forward and backward, and the feature-distance loss with its
// gradient (perceptual.py:155-167: nn.L1Loss / nn.MSELoss, mean reduction).
// NHWC activations of the compute dtype, 16 B per lane; HBM-bound, one pass each.
#include "fen_common.h"

namespace {

inline int nblk(size_t n, int t = 256) { return (int)((n + t - 1) / t); }

// y[b][h][w][c] = max over the 2x2 window at (2h, 2w) (torch max_pool2d(2, 2))
template <typename T>
__global__ __launch_bounds__(256) void k_maxpool2(int B, int Ho, int Wo, int C, const T* __restrict__ x,
                                                  T* __restrict__ y) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * Ho * Wo * G) return;
    const int g = (int)(i % G);
    const size_t po = i / G;
    const int wo = (int)(po % Wo), ho = (int)((po / Wo) % Ho), b = (int)(po / ((size_t)Wo * Ho));
    const int W = 2 * Wo;
    float m[V], v[V];
    const size_t p00 = ((size_t)(b * 2 * Ho + 2 * ho) * W + 2 * wo) * C + g * V;
    unpack16<T>(*(const uint4*)(x + p00), m);
    const size_t offs[3] = {(size_t)C, (size_t)W * C, (size_t)W * C + C};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        unpack16<T>(*(const uint4*)(x + p00 + offs[k]), v);
#pragma unroll
        for (int j = 0; j < V; ++j) m[j] = v[j] > m[j] ? v[j] : m[j];
    }
    *(uint4*)(y + po * C + g * V) = pack16<T>(m);
}

// dx = max-pool backward of dy through the pre-pool activation a (torch routes each window's
// gradient to its FIRST maximum in (0,0),(0,1),(1,0),(1,1) order), times the ReLU mask
// [a > 0] of the ReLU that produced a (torchvision: conv -> ReLU -> pool); other taps 0.
template <typename T>
__global__ __launch_bounds__(256) void k_maxpool2_bwd_relu(int B, int Ho, int Wo, int C, const T* __restrict__ dy,
                                                           const T* __restrict__ a, T* __restrict__ dx) {
    constexpr int V = 16 / sizeof(T);
    const int G = C / V;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * Ho * Wo * G) return;
    const int g = (int)(i % G);
    const size_t po = i / G;
    const int wo = (int)(po % Wo), ho = (int)((po / Wo) % Ho), b = (int)(po / ((size_t)Wo * Ho));
    const int W = 2 * Wo;
    const size_t p00 = ((size_t)(b * 2 * Ho + 2 * ho) * W + 2 * wo) * C + g * V;
    const size_t offs[4] = {0, (size_t)C, (size_t)W * C, (size_t)W * C + C};
    float av[4][V], d[V];
#pragma unroll
    for (int k = 0; k < 4; ++k) unpack16<T>(*(const uint4*)(a + p00 + offs[k]), av[k]);
    unpack16<T>(*(const uint4*)(dy + po * C + g * V), d);
    int arg[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        float m = av[0][j];
        int am = 0;
#pragma unroll
        for (int k = 1; k < 4; ++k)
            if (av[k][j] > m) { m = av[k][j]; am = k; }
        arg[j] = m > 0.f ? am : -1;               // a = ReLU output: max <= 0 means no gradient
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = arg[j] == k ? d[j] : 0.f;
        *(uint4*)(dx + p00 + offs[k]) = pack16<T>(o);
    }
}

// Feature distance between the two halves of one batch: f = [pred (nimg images); target
// (nimg images)], n = nimg * per-image elements.  part[block] = sum |p - t| (L1) or
// sum (p - t)^2 (L2) over the block's elements (fixed order), and the pred-half gradient
//   g = (accumulate ? g : 0) + scale * sign(p - t)       (L1; sign(0) = 0 as torch)
//   g = (accumulate ? g : 0) + scale * 2 (p - t)          (L2)
// with scale = layer weight / n.  256 threads x V elements per iteration, grid-stride.
constexpr int FL_BLOCKS = 1024;
template <typename T>
__global__ __launch_bounds__(256) void k_feat_loss(size_t n, const T* __restrict__ f, int l2, float scale,
                                                   T* __restrict__ g, int accumulate, float* __restrict__ part) {
    constexpr int V = 16 / sizeof(T);
    __shared__ float red[256];
    const T* p = f;
    const T* t = f + n;
    float acc = 0.f;
    const size_t nv = n / V;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
        float pv[V], tv[V], gv[V], go[V];
        unpack16<T>(*(const uint4*)(p + i * V), pv);
        unpack16<T>(*(const uint4*)(t + i * V), tv);
        if (accumulate) unpack16<T>(*(const uint4*)(g + i * V), gv);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float dlt = pv[j] - tv[j];
            float gr;
            if (l2) {
                acc += dlt * dlt;
                gr = 2.f * dlt;
            } else {
                acc += fabsf(dlt);
                gr = dlt > 0.f ? 1.f : (dlt < 0.f ? -1.f : 0.f);
            }
            go[j] = (accumulate ? gv[j] : 0.f) + scale * gr;
        }
        *(uint4*)(g + i * V) = pack16<T>(go);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

}  // namespace

#define STREAM ((hipStream_t)stream)

extern "C" int fen_maxpool2(int dtype, int B, int H, int W, int C, const void* x, void* y, void* stream) {
    if (!x || !y || B <= 0 || (H | W) & 1 || H <= 0 || W <= 0 || C % 8) return FEN_EINVAL;
    const size_t n = (size_t)B * (H / 2) * (W / 2) * (C / (dtype == FEN_F32 ? 4 : 8));
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_maxpool2<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C, (const bf16*)x,
                           (bf16*)y);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_maxpool2<f16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C, (const f16*)x,
                           (f16*)y);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_maxpool2<float>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C, (const float*)x,
                           (float*)y);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_maxpool2_bwd_relu(int dtype, int B, int H, int W, int C, const void* dy, const void* a, void* dx,
                                     void* stream) {
    if (!dy || !a || !dx || B <= 0 || (H | W) & 1 || H <= 0 || W <= 0 || C % 8) return FEN_EINVAL;
    const size_t n = (size_t)B * (H / 2) * (W / 2) * (C / (dtype == FEN_F32 ? 4 : 8));
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_maxpool2_bwd_relu<bf16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C,
                           (const bf16*)dy, (const bf16*)a, (bf16*)dx);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_maxpool2_bwd_relu<f16>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C,
                           (const f16*)dy, (const f16*)a, (f16*)dx);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_maxpool2_bwd_relu<float>, dim3(nblk(n)), dim3(256), 0, STREAM, B, H / 2, W / 2, C,
                           (const float*)dy, (const float*)a, (float*)dx);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// mean |pred - target| over fp32 tensors (nn.L1Loss, combined.py:38-47 / the trainer's fallback
// F.l1_loss): part[blk] = sum |p - t| of the block's elements (fixed order); with grad:
// grad = scale * (gs ? *gs : 1) * sign(p - t) (gs: the upstream gradient, read on the device)
__global__ __launch_bounds__(256) void k_l1(size_t n, const float* __restrict__ p, const float* __restrict__ t,
                                            const float* __restrict__ gs, float scale, float* __restrict__ g,
                                            float* __restrict__ part) {
    __shared__ float red[256];
    const float sc = g ? scale * (gs ? gs[0] : 1.f) : 0.f;
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float d = p[i] - t[i];
        acc += fabsf(d);
        if (g) g[i] = d > 0.f ? sc : (d < 0.f ? -sc : 0.f);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

extern "C" int fen_l1_loss(size_t n, const float* pred, const float* target, const float* gscale, float scale,
                           float* grad, float* part, void* stream) {
    if (!pred || !target || !part || n == 0) return FEN_EINVAL;
    hipLaunchKernelGGL(k_l1, dim3(FL_BLOCKS), dim3(256), 0, STREAM, n, pred, target, gscale, scale, grad, part);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

extern "C" int fen_feat_loss_parts(void) { return FL_BLOCKS; }

extern "C" int fen_feat_loss(int dtype, size_t n, const void* f, int l2, float scale, void* g, int accumulate,
                             float* part, void* stream) {
    if (!f || !g || !part || n == 0 || n % 8) return FEN_EINVAL;
    if (dtype == FEN_BF16)
        hipLaunchKernelGGL(k_feat_loss<bf16>, dim3(FL_BLOCKS), dim3(256), 0, STREAM, n, (const bf16*)f, l2, scale,
                           (bf16*)g, accumulate, part);
    else if (dtype == FEN_F16)
        hipLaunchKernelGGL(k_feat_loss<f16>, dim3(FL_BLOCKS), dim3(256), 0, STREAM, n, (const f16*)f, l2, scale,
                           (f16*)g, accumulate, part);
    else if (dtype == FEN_F32)
        hipLaunchKernelGGL(k_feat_loss<float>, dim3(FL_BLOCKS), dim3(256), 0, STREAM, n, (const float*)f, l2, scale,
                           (float*)g, accumulate, part);
    else
        return FEN_EINVAL;
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// HR batch preparation on the device (reference src/data/transforms.py:173-279 train-mode
// pairs transform + to_tensor 260-279; scripts/train.py:174-198 defaults): uint8 HWC crops
// (gathered on the host into pinned staging, copied async) -> horizontal flip -> colour jitter
// (brightness, contrast around the image mean, uint8 quantisation, HSV saturation through an
// 8-bit RGB->HSV->RGB round trip) -> /255 -> NCHW fp32, written straight into the training
// engine's HR buffer.  Per-image parameters come from the host (the reference draws them with
// np.random per sample).
//
// The HSV round trip follows OpenCV's published 8-bit algorithm (RGB2HSV_b fixed-point with
// hsv_shift 12 and its division tables, H in [0,180); HSV2RGB_b via float sectors, cvRound):
// cv2 is absent offline, so that step's parity is UNPINNED; flip, brightness, contrast and the
// uint8 quantisation follow the reference's numpy code exactly (tests/test_gpu_augment.py).
#include "fen_common.h"

namespace {

struct AugParam {
    int flip, jitter;
    float brightness, contrast, saturation;
    int rot;            // np.rot90(k) after the flip (k = 0..3)
};

// per-image sum of the uint8 crop (exact in int64) -> the contrast mean
__global__ __launch_bounds__(256) void k_img_sum(int P, const unsigned char* __restrict__ src,
                                                 long long* __restrict__ sums) {
    __shared__ long long red[256];
    const int b = blockIdx.x;
    const size_t n = (size_t)P * P * 3;
    const unsigned char* s = src + (size_t)b * n;
    long long acc = 0;
    for (size_t i = threadIdx.x * 4; i < n; i += 256 * 4) {
        if (i + 4 <= n) {
            const unsigned w = *(const unsigned*)(s + i);
            acc += (w & 255) + ((w >> 8) & 255) + ((w >> 16) & 255) + (w >> 24);
        } else {
            for (size_t k = i; k < n; ++k) acc += s[k];
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[b] = red[0];
}

__device__ __forceinline__ int cv_round(double x) { return (int)rint(x); }

// OpenCV RGB2HSV_b (hrange 180), one pixel
__device__ __forceinline__ void rgb2hsv8(int r, int g, int b, int& h, int& s, int& v) {
    constexpr int shift = 12;
    v = max(max(b, g), r);
    const int vmin = min(min(b, g), r);
    const int diff = v - vmin;
    const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    const int sdiv = v ? cv_round((double)(255 << shift) / v) : 0;
    const int hdiv = diff ? cv_round((double)(180 << shift) / (6.0 * diff)) : 0;
    s = (diff * sdiv + (1 << (shift - 1))) >> shift;
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + (~vg & (r - g + 4 * diff))));
    h = (h * hdiv + (1 << (shift - 1))) >> shift;
    h += h < 0 ? 180 : 0;
}

// OpenCV HSV2RGB_b (hrange 180), one pixel
__device__ __forceinline__ void hsv2rgb8(int hi, int si, int vi, int& r, int& g, int& b) {
    float h = (float)hi, s = si * (1.f / 255.f), v = vi * (1.f / 255.f);
    float fb, fg, fr;
    if (s == 0.f) {
        fb = fg = fr = v;
    } else {
        h *= 6.f / 180.f;
        while (h < 0.f) h += 6.f;
        while (h >= 6.f) h -= 6.f;
        int sector = (int)floorf(h);
        h -= sector;
        if ((unsigned)sector >= 6u) { sector = 0; h = 0.f; }
        const float tab[4] = {v, v * (1.f - s), v * (1.f - s * h), v * (1.f - s * (1.f - h))};
        const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        fb = tab[sd[sector][0]];
        fg = tab[sd[sector][1]];
        fr = tab[sd[sector][2]];
    }
    b = min(max(cv_round(fb * 255.f), 0), 255);
    g = min(max(cv_round(fg * 255.f), 0), 255);
    r = min(max(cv_round(fr * 255.f), 0), 255);
}

// thread per output pixel; out NCHW fp32 [B,3,P,P]
__global__ __launch_bounds__(256) void k_augment(int B, int P, const unsigned char* __restrict__ src,
                                                 const AugParam* __restrict__ prm, const long long* __restrict__ sums,
                                                 float* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t npx = (size_t)P * P;
    if (i >= (size_t)B * npx) return;
    const int b = (int)(i / npx);
    const int y = (int)((i % npx) / P), x = (int)(i % P);
    const AugParam a = prm[b];
    // output (y, x) of rot90_k(F), F = the flipped crop; np.rot90 turns counter-clockwise
    int fy = y, fx = x;
    if (a.rot == 1) { fy = x; fx = P - 1 - y; }
    else if (a.rot == 2) { fy = P - 1 - y; fx = P - 1 - x; }
    else if (a.rot == 3) { fy = P - 1 - x; fx = y; }
    const int xs = a.flip ? P - 1 - fx : fx;
    const unsigned char* px = src + (((size_t)b * P + fy) * P + xs) * 3;
    int c[3] = {px[0], px[1], px[2]};
    if (a.jitter) {
        // img_float = img / 255 * brightness; mean over the image; (f - mean) * contrast + mean;
        // clip(f * 255, 0, 255).astype(uint8) -- float32 arithmetic as numpy does it
        const float mean = (float)((double)sums[b] / (255.0 * 3.0 * (double)npx) * (double)a.brightness);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float f = (float)c[k] / 255.f * a.brightness;
            f = (f - mean) * a.contrast + mean;
            f = fminf(fmaxf(f * 255.f, 0.f), 255.f);
            c[k] = (int)f;                                   // astype(uint8): truncation
        }
        // cvtColor(RGB2HSV) -> float32 -> S *= saturation -> clip -> astype(uint8) -> HSV2RGB
        int h, s, v;
        rgb2hsv8(c[0], c[1], c[2], h, s, v);
        const int s2 = (int)fminf(fmaxf((float)s * a.saturation, 0.f), 255.f);
        hsv2rgb8(h, s2, v, c[0], c[1], c[2]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) out[((size_t)b * 3 + k) * npx + (size_t)y * P + x] = (float)c[k] / 255.f;
}

}  // namespace

#define STREAM ((hipStream_t)stream)

// params: B records of {int flip, int jitter, float brightness, contrast, saturation, int rot}
extern "C" int fen_augment_u8(int B, int P, const void* src_u8, const void* params, long long* sums, float* out,
                              void* stream) {
    if (!src_u8 || !params || !sums || !out || B <= 0 || P <= 0 || (P & 1)) return FEN_EINVAL;
    hipLaunchKernelGGL(k_img_sum, dim3(B), dim3(256), 0, STREAM, P, (const unsigned char*)src_u8, sums);
    FEN_CHECK_LAUNCH();
    const size_t n = (size_t)B * P * P;
    hipLaunchKernelGGL(k_augment, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, STREAM, B, P,
                       (const unsigned char*)src_u8, (const AugParam*)params, sums, out);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

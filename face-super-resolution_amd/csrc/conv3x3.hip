// 3x3 / stride 1 / pad 1 convolution on NHWC activations as an implicit GEMM on MFMA (gfx950).
//
// Replaces every nn.Conv2d(k=3, pad=1) forward of the hot path (reference blocks.py:123-131,
// 182-183, 211-214; custom.py:109-112, 121-124) and, given flipped/transposed weights
// (fen_pack_conv_w mode 2), the data-gradient of each of them.
//
// Block = 256 threads (4 waves), output tile = 16x16 pixels x COT output channels.
//   D[co][px] = sum_k W[co][k] * X[k][px],  k = (tap, ci):  A = weights, B = pixels.
//   Each wave owns 4 output rows (4 x 16 px) x COT co -> MT*4 16x16 accumulators.
// LDS: the 18x18-pixel input halo of one 128-B channel panel (41.5 KB, XOR-swizzled rows)
//      + two 128-B-row weight tiles [COT][panel] (one per tap, double buffered, T14 split
//      issue-early / write-late).  57.9 KB at COT=64 -> 2 blocks (8 waves) per CU.
// Epilogue fuses bias, residual adds, PReLU (fwd) or PReLU-backward (dgrad), PixelShuffle /
// inverse-PixelShuffle stores, SE global-average-pool partials, and for conv_last the
// bicubic skip + eval clamp + L1-loss gradient.  bf16 tiles leave through LDS as full
// 128-B rows (coalesced 16-B stores).
#include "fen_common.h"

namespace {

constexpr int HALO = 18;
constexpr int HP = HALO * HALO;        // 324 halo pixels
constexpr int HALO_BYTES = HP * 128;   // 41472

template <typename T, int COT>
__global__ __launch_bounds__(256, 2) void k_conv3x3(const fen_conv_desc d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* halo = smem;
    char* wbuf = smem + HALO_BYTES;
    constexpr int MT = COT / 16;
    constexpr int CK = Tr<T>::CK;
    constexpr int WCH = COT * 8;               // 16-B weight chunks per (tap, panel)
    constexpr int WPT = (WCH + 255) / 256;     // per thread

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q = lane >> 4, c16 = lane & 15;
    const int H = d.H, W = d.W, Cin = d.Cin, Cout = d.Cout;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int b = blockIdx.x / tpi, tile = blockIdx.x - b * tpi;
    const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
    const int co0 = blockIdx.y * COT;
    const int coutp = (Cout + 15) & ~15;
    const char* xb = (const char*)d.x;
    const char* wb = (const char*)d.w;
    const size_t xrow = (size_t)Cin * sizeof(T);
    const size_t wrow = (size_t)Cin * sizeof(T);

    f32x4 acc[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int npan = Cin / CK;
    for (int pn = 0; pn < npan; ++pn) {
        // ---- stage the input halo of panel pn (zero padding outside the image) ----
        for (int i = tid; i < HP * 8; i += 256) {
            const int p = i >> 3, ch = i & 7;
            const int hr = p / HALO, hc = p - hr * HALO;
            const int gh = h0 + hr - 1, gw = w0 + hc - 1;
            uint4 v = make_uint4(0, 0, 0, 0);
            if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W)
                v = *(const uint4*)(xb + ((size_t)(b * H + gh) * W + gw) * xrow + pn * 128 + ch * 16);
            *(uint4*)(halo + swz(p, ch)) = v;
        }
        uint4 wr[WPT];
        auto load_w = [&](int tap) {
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const int i = tid + j * 256;
                if (i < WCH) {
                    const int r = i >> 3, ch = i & 7;
                    wr[j] = *(const uint4*)(wb + (size_t)(tap * coutp + co0 + r) * wrow + pn * 128 + ch * 16);
                }
            }
        };
        auto store_w = [&](char* dst) {
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const int i = tid + j * 256;
                if (i < WCH) *(uint4*)(dst + swz(i >> 3, i & 7)) = wr[j];
            }
        };
        load_w(0);
        store_w(wbuf);
        __syncthreads();
        for (int tap = 0; tap < 9; ++tap) {
            if (tap < 8) load_w(tap + 1);      // issue early, write after the MFMAs
            const char* wt = wbuf + (tap & 1) * COT * 128;
            const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int chunk = kk * 4 + q;
                uint4 A[MT], Bf[4];
#pragma unroll
                for (int m = 0; m < MT; ++m) A[m] = *(const uint4*)(wt + swz(m * 16 + c16, chunk));
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const int p = (wave * 4 + n + kh) * HALO + c16 + kw;
                    Bf[n] = *(const uint4*)(halo + swz(p, chunk));
                }
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int n = 0; n < 4; ++n) mma16<T>(acc[m][n], A[m], Bf[n]);
            }
            if (tap < 8) store_w(wbuf + ((tap + 1) & 1) * COT * 128);
            __syncthreads();
        }
    }

    // ------------------------------- epilogue -------------------------------
    const int epi = d.epi;
    float* red = (float*)wbuf;                 // [4 waves][COT] (LDS is free after the loop)
    const int w_ = w0 + c16;

    if (epi & FEN_EPI_LAST) {
        // conv_last: rows co = 4q + r; only co < Cout (3) are real.  One bicubic sample per
        // lane: lane (q, c16) computes channel q of pixel c16, then lanes of q == 0 gather.
        const int Hs = H / d.scale, Ws = W / d.scale;
        const float inv = 1.0f / (float)d.scale;
        float lsum = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int h = h0 + wave * 4 + n;
            const bool valid = h < H && w_ < W;
            float bic = 0.f;
            if (valid && q < Cout)
                bic = bicubic_sample(d.lr + ((size_t)b * Cout + q) * Hs * Ws, Hs, Ws, h, w_, inv);
            float bq[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bq[r] = __shfl(bic, r * 16 + c16, 64);
            float g4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = q * 4 + r;
                if (valid && co < Cout) {
                    float v = acc[0][n][r] + ((epi & FEN_EPI_BIAS) ? d.bias[co] : 0.f) + bq[r];
                    if (d.clamp) v = fminf(fmaxf(v, 0.f), 1.f);
                    const size_t oi = (((size_t)b * Cout + co) * H + h) * W + w_;
                    if (d.y) ((float*)d.y)[oi] = v;
                    if (d.hr) {
                        const float diff = v - d.hr[oi];
                        lsum += fabsf(diff);
                        g4[r] = diff > 0.f ? d.l1_scale : (diff < 0.f ? -d.l1_scale : 0.f);
                    }
                }
            }
            if (d.hr && d.dout && valid)
                st4<T>((char*)d.dout + (((size_t)(b * H + h) * W + w_) * 16 + q * 4) * sizeof(T), g4);
        }
        if (d.hr && d.loss_part) {
            lsum = wave_sum(lsum);
            if (lane == 0) red[wave] = lsum;
            __syncthreads();
            if (tid == 0) d.loss_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
        }
        return;
    }

    const bool shuf = epi & FEN_EPI_SHUFFLE;
    const bool unshuf = epi & FEN_EPI_UNSHUFFLE;
    const int Cq = Cout >> 2;
    float psum[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) psum[m][r] = 0.f;

    // pass 1: elementwise epilogue in registers (acc <- pre-activation value)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int cob = co0 + m * 16 + q * 4;      // first of 4 consecutive (packed) channels
        float bias4[4] = {0.f, 0.f, 0.f, 0.f};
        if (epi & FEN_EPI_BIAS) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int cp = cob + r;
                const int co = shuf ? 4 * (cp % Cq) + cp / Cq : cp;
                bias4[r] = cob < Cout ? d.bias[co] : 0.f;
            }
        }
        float al4[4] = {0.f, 0.f, 0.f, 0.f};
        if ((epi & FEN_EPI_PRELU_BWD) && cob < Cout) {
#pragma unroll
            for (int r = 0; r < 4; ++r) al4[r] = d.alpha[cob + r];
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int h = h0 + wave * 4 + n;
            const bool valid = h < H && w_ < W && cob < Cout;
            const size_t oi = ((size_t)(b * H + h) * W + w_) * Cout + cob;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[m][n][r] + bias4[r];
            if (valid) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    if (d.res[k]) {
                        float rv[4];
                        ld4<T>((const char*)d.res[k] + oi * sizeof(T), rv);
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += rv[r];
                    }
                }
                if (epi & FEN_EPI_PRELU_BWD) {
                    float pv[4];
                    ld4<T>((const char*)d.pre_in + oi * sizeof(T), pv);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        psum[m][r] += pv[r] > 0.f ? 0.f : v[r] * pv[r];
                        v[r] = pv[r] > 0.f ? v[r] : v[r] * al4[r];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m][n][r] = v[r];
            if ((epi & FEN_EPI_POOL) && valid) {
#pragma unroll
                for (int r = 0; r < 4; ++r) psum[m][r] += v[r];
            }
        }
    }

    // per-channel partial sums (SE pool or PReLU dalpha): 16-lane butterfly, then across waves
    if (epi & (FEN_EPI_POOL | FEN_EPI_PRELU_BWD)) {
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float s = group16_sum(psum[m][r]);
                if (c16 == 0) red[wave * COT + m * 16 + q * 4 + r] = s;
            }
        __syncthreads();
        if (tid < COT && co0 + tid < Cout)
            d.part[(size_t)blockIdx.x * Cout + co0 + tid] =
                red[tid] + red[COT + tid] + red[2 * COT + tid] + red[3 * COT + tid];
    }

    const bool prelu = epi & FEN_EPI_PRELU;
    // value actually stored for output k (0: y_pre, 1: y)
    auto final_v = [&](float v, int cp, int k) -> float {
        if (k == 1 && prelu) {
            const float a = d.alpha[shuf ? (cp % Cq) : cp];
            return v > 0.f ? v : a * v;
        }
        return v;
    };

    if constexpr (sizeof(T) == 2 && COT == 64) {
        // ---- bf16: stage the 256 x 64 tile in LDS, leave as full 128-B rows ----
        char* st = halo;
        for (int k = 0; k < 2; ++k) {
            void* dst = k == 0 ? d.y_pre : d.y;
            if (k == 0 && (!prelu || !dst)) continue;
            __syncthreads();
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const int cl = m * 16 + q * 4;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const int px = (wave * 4 + n) * 16 + c16;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = final_v(acc[m][n][r], co0 + cl + r, k);
                    st4<bf16>(st + swz(px, cl >> 3) + (q & 1) * 8, v);
                }
            }
            __syncthreads();
            if (!unshuf) {
                for (int i = tid; i < 256 * 8; i += 256) {
                    const int px = i >> 3, ch = i & 7;
                    const int h = h0 + (px >> 4), w = w0 + (px & 15);
                    if (h >= H || w >= W) continue;
                    const uint4 v = *(const uint4*)(st + swz(px, ch));
                    size_t o;
                    if (shuf) {
                        const int cp = co0 + ch * 8, t = cp / Cq, c = cp % Cq;
                        o = ((size_t)(b * 2 * H + 2 * h + (t >> 1)) * (2 * W) + 2 * w + (t & 1)) * Cq + c;
                    } else {
                        o = ((size_t)(b * H + h) * W + w) * Cout + co0 + ch * 8;
                    }
                    *(uint4*)((char*)dst + o * 2) = v;
                }
            } else {
                // du[b][h/2][w/2][4*co + 2*(h&1) + (w&1)]: 8x8 du pixels x 4*COT channels
                const int Hh = H >> 1, Wh = W >> 1;
                for (int i = tid; i < 64 * 32; i += 256) {
                    const int dp = i >> 5, kq = i & 31;
                    const int hh = dp >> 3, ww = dp & 7;
                    const int gh = (h0 >> 1) + hh, gw = (w0 >> 1) + ww;
                    if (gh >= Hh || gw >= Wh) continue;
                    unsigned short e[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int cl = 2 * kq + (j >> 2), t = j & 3;
                        const int px = (2 * hh + (t >> 1)) * 16 + 2 * ww + (t & 1);
                        e[j] = *(const unsigned short*)(st + swz(px, cl >> 3) + (cl & 7) * 2);
                    }
                    uint4 u;
                    u.x = e[0] | ((unsigned)e[1] << 16);
                    u.y = e[2] | ((unsigned)e[3] << 16);
                    u.z = e[4] | ((unsigned)e[5] << 16);
                    u.w = e[6] | ((unsigned)e[7] << 16);
                    const size_t o = ((size_t)(b * Hh + gh) * Wh + gw) * (4 * Cout) + 4 * co0 + 8 * kq;
                    *(uint4*)((char*)dst + o * 2) = u;
                }
            }
        }
    } else {
        // ---- direct stores from registers (f32, or bf16 with COT != 64) ----
        for (int k = 0; k < 2; ++k) {
            void* dst = k == 0 ? d.y_pre : d.y;
            if (k == 0 && (!prelu || !dst)) continue;
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const int cob = co0 + m * 16 + q * 4;
                if (cob >= Cout) continue;
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const int h = h0 + wave * 4 + n;
                    if (h >= H || w_ >= W) continue;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = final_v(acc[m][n][r], cob + r, k);
                    if (shuf) {
                        const int t = cob / Cq, c = cob % Cq;
                        const size_t o = ((size_t)(b * 2 * H + 2 * h + (t >> 1)) * (2 * W) + 2 * w_ + (t & 1)) * Cq + c;
                        st4<T>((char*)dst + o * sizeof(T), v);
                    } else if (unshuf) {
                        const int Hh = H >> 1, Wh = W >> 1, t = 2 * (h & 1) + (w_ & 1);
                        const size_t o = ((size_t)(b * Hh + (h >> 1)) * Wh + (w_ >> 1)) * (4 * Cout) + t;
#pragma unroll
                        for (int r = 0; r < 4; ++r) ((T*)dst)[o + 4 * (cob + r)] = fromf<T>(v[r]);
                    } else {
                        const size_t o = ((size_t)(b * H + h) * W + w_) * Cout + cob;
                        st4<T>((char*)dst + o * sizeof(T), v);
                    }
                }
            }
        }
    }
}

template <typename T, int COT>
int launch_conv(const fen_conv_desc* d, hipStream_t s) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int coutp = (d->Cout + 15) & ~15;
    dim3 grid(d->B * tpi, coutp / COT);
    const size_t lds = HALO_BYTES + 2 * COT * 128;
    hipLaunchKernelGGL((k_conv3x3<T, COT>), grid, dim3(256), lds, s, *d);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

}  // namespace

extern "C" int fen_conv3x3(const fen_conv_desc* d, void* stream) {
    if (!d || !d->x || !d->w || d->B <= 0 || d->H <= 0 || d->W <= 0 || d->Cin <= 0 || d->Cout <= 0)
        return FEN_EINVAL;
    const int CK = d->dtype == FEN_BF16 ? 64 : 32;
    if (d->dtype != FEN_F32 && d->dtype != FEN_BF16) return FEN_EINVAL;
    if (d->Cin % CK) return FEN_EUNSUPPORTED;
    const int epi = d->epi;
    if ((epi & FEN_EPI_BIAS) && !d->bias) return FEN_EINVAL;
    if ((epi & (FEN_EPI_PRELU | FEN_EPI_PRELU_BWD)) && !d->alpha) return FEN_EINVAL;
    if ((epi & FEN_EPI_PRELU_BWD) && !d->pre_in) return FEN_EINVAL;
    if ((epi & (FEN_EPI_POOL | FEN_EPI_PRELU_BWD)) && !d->part) return FEN_EINVAL;
    if ((epi & FEN_EPI_POOL) && (epi & FEN_EPI_PRELU_BWD)) return FEN_EUNSUPPORTED;
    if ((epi & (FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE)) == (FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE))
        return FEN_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    if (epi & FEN_EPI_LAST) {
        if (d->Cout > 4 || !d->lr || d->scale <= 0 || d->H % d->scale || d->W % d->scale) return FEN_EINVAL;
        if (epi & ~(FEN_EPI_LAST | FEN_EPI_BIAS)) return FEN_EUNSUPPORTED;
        return d->dtype == FEN_BF16 ? launch_conv<bf16, 16>(d, s) : launch_conv<float, 16>(d, s);
    }
    if (!d->y) return FEN_EINVAL;
    if (epi & FEN_EPI_SHUFFLE) {
        if (d->Cout % 64) return FEN_EUNSUPPORTED;
        if (epi & (FEN_EPI_PRELU_BWD | FEN_EPI_POOL) || d->res[0] || d->res[1] || d->res[2])
            return FEN_EUNSUPPORTED;
    }
    if ((epi & FEN_EPI_UNSHUFFLE) && ((d->H | d->W) & 1)) return FEN_EINVAL;
    if (d->Cout % 64 == 0)
        return d->dtype == FEN_BF16 ? launch_conv<bf16, 64>(d, s) : launch_conv<float, 64>(d, s);
    if (d->Cout % 16 == 0)
        return d->dtype == FEN_BF16 ? launch_conv<bf16, 16>(d, s) : launch_conv<float, 16>(d, s);
    return FEN_EUNSUPPORTED;
}

// Weight gradient of the 3x3 convs (autograd of nn.Conv2d on the hot path, reference
// trainer.py:482-485 -> blocks.py / custom.py convs) as a split-K GEMM on MFMA (gfx950).
//
//   dW[co][tap][ci] = sum_px dy[px][co] * x[px + off(tap)][ci]        (K = pixels)
//   db[co]          = sum_px dy[px][co]                               (one extra MFMA vs ones)
//
// Block = 9 waves, wave w owns tap w: a 16x16-pixel dy tile [256 px][COT] and the 18x18
// input halo [324 px][64 ci] are staged in LDS (XOR-swizzled 128-B panel rows) and every
// wave reads the same dy fragments and its own tap-shifted input fragments.  bf16 uses the
// gfx950 transposed LDS read ds_read_b64_tr_b16 to build k=pixel fragments from the
// channels-last image; f32 uses 16x16x4 f32 MFMAs with ds_read_b32 operands.
// Each block accumulates a chunk of pixel tiles in registers and writes one fp32 slab; a
// second kernel reduces the slabs in fixed order (bitwise reproducible) straight into
// the reference OIHW layout.
#include "fen_common.h"

namespace {

constexpr int HALO = 18;
constexpr int HP = HALO * HALO;
constexpr int PANEL_HALO = HP * 128;   // 41472 B
constexpr int PANEL_TILE = 256 * 128;  // 32768 B

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T>
__device__ __forceinline__ int pan_off(int p, int c, int pbytes) {
    constexpr int CK = Tr<T>::CK, EPC = Tr<T>::EPC;
    return (c / CK) * pbytes + swz(p, (c % CK) / EPC) + (c % EPC) * (int)sizeof(T);
}

template <typename T, int COT>
__global__ __launch_bounds__(576, 1) void k_wgrad(const fen_wgrad_desc d, int tpc, float* part, float* dbpart) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int CK = Tr<T>::CK;
    constexpr int NPX = 64 / CK;                                  // panels of the 64-ci halo
    constexpr int YCH = COT * (int)sizeof(T) / 16;                // 16-B chunks per dy pixel
    char* hx = smem;                                              // [NPX][324 px][128 B]
    char* ty = smem + NPX * PANEL_HALO;                           // [NPY][256 px][128 B]
    constexpr int MT = COT / 16;

    const int tid = threadIdx.x, lane = tid & 63, tap = tid >> 6;
    const int q = lane >> 4, c16 = lane & 15;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int H = d.H, W = d.W, Cin = d.Cin, Cout = d.Cout;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int ntiles = d.B * tpi;
    const int co0 = blockIdx.y * COT, ci0 = blockIdx.z * 64;
    const int t_begin = blockIdx.x * tpc, t_end = min(t_begin + tpc, ntiles);

    f32x4 acc[MT][4];
    f32x4 accb[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        accb[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const bool do_db = (tap == 0) && (blockIdx.z == 0) && dbpart != nullptr;

    for (int tt = t_begin; tt < t_end; ++tt) {
        const int b = tt / tpi, tile = tt - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        __syncthreads();
        // stage x halo (64 channels from ci0) and the dy tile (COT channels from co0)
        for (int i = tid; i < HP * 8 * NPX; i += 576) {
            const int pn = i / (HP * 8), j = i - pn * HP * 8;
            const int p = j >> 3, ch = j & 7;
            const int hr = p / HALO, hc = p - hr * HALO;
            const int gh = h0 + hr - 1, gw = w0 + hc - 1;
            uint4 v = make_uint4(0, 0, 0, 0);
            if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W)
                v = *(const uint4*)((const char*)d.x +
                                    (((size_t)(b * H + gh) * W + gw) * Cin + ci0 + pn * CK) * sizeof(T) + ch * 16);
            *(uint4*)(hx + pn * PANEL_HALO + swz(p, ch)) = v;
        }
        for (int i = tid; i < 256 * YCH; i += 576) {
            const int p = i / YCH, j = i - p * YCH;
            const int pn = j >> 3, ch = j & 7;
            const int gh = h0 + (p >> 4), gw = w0 + (p & 15);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (gh < H && gw < W)
                v = *(const uint4*)((const char*)d.dy +
                                    (((size_t)(b * H + gh) * W + gw) * Cout + co0) * sizeof(T) + j * 16);
            *(uint4*)(ty + pn * PANEL_TILE + swz(p, ch)) = v;
        }
        __syncthreads();

        if constexpr (sizeof(T) == 2) {
            // 8 k-steps of 32 pixels: step s covers tile rows 2s, 2s+1
            const int qq = c16 >> 2, pp = c16 & 3;
            const uint4 ones = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
#pragma unroll 2
            for (int s = 0; s < 8; ++s) {
                uint4 A[MT], Bf[4];
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int k = 8 * q + 4 * half + qq;                 // pixel of this lane's row
                    const int prow = 2 * s + (k >> 4), pcol = k & 15;
                    const int py = prow * 16 + pcol;
                    const int ph = (prow + kh) * HALO + pcol + kw;
#pragma unroll
                    for (int m = 0; m < MT; ++m) {
                        const int c = m * 16 + 4 * pp;
                        s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s16x4*)(ty + swz(py, c >> 3) + (c & 7) * 2));
                        const uint2 u = __builtin_bit_cast(uint2, v);
                        if (half == 0) { A[m].x = u.x; A[m].y = u.y; } else { A[m].z = u.x; A[m].w = u.y; }
                    }
#pragma unroll
                    for (int n = 0; n < 4; ++n) {
                        const int c = n * 16 + 4 * pp;
                        s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s16x4*)(hx + swz(ph, c >> 3) + (c & 7) * 2));
                        const uint2 u = __builtin_bit_cast(uint2, v);
                        if (half == 0) { Bf[n].x = u.x; Bf[n].y = u.y; } else { Bf[n].z = u.x; Bf[n].w = u.y; }
                    }
                }
#pragma unroll
                for (int m = 0; m < MT; ++m) {
#pragma unroll
                    for (int n = 0; n < 4; ++n) mma16<bf16>(acc[m][n], A[m], Bf[n]);
                    if (do_db) mma16<bf16>(accb[m], A[m], ones);
                }
            }
        } else {
            // 64 k-steps of 4 pixels (16x16x4 f32): lane group q is the k index
#pragma unroll 4
            for (int s = 0; s < 64; ++s) {
                const int prow = s >> 2, pcol = (s & 3) * 4 + q;
                const int py = prow * 16 + pcol;
                const int ph = (prow + kh) * HALO + pcol + kw;
                float a[MT], bv[4];
#pragma unroll
                for (int m = 0; m < MT; ++m) a[m] = *(const float*)(ty + pan_off<float>(py, m * 16 + c16, PANEL_TILE));
#pragma unroll
                for (int n = 0; n < 4; ++n) bv[n] = *(const float*)(hx + pan_off<float>(ph, n * 16 + c16, PANEL_HALO));
#pragma unroll
                for (int m = 0; m < MT; ++m) {
#pragma unroll
                    for (int n = 0; n < 4; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bv[n], acc[m][n], 0, 0, 0);
                    if (do_db) accb[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], 1.0f, accb[m], 0, 0, 0);
                }
            }
        }
    }

    // slab store: lane holds D[co = m*16 + 4q + r][ci = n*16 + c16]
    float* slab = part + (size_t)blockIdx.x * 9 * Cout * Cin;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + m * 16 + q * 4 + r, ci = ci0 + n * 16 + c16;
                slab[((size_t)tap * Cout + co) * Cin + ci] = acc[m][n][r];
            }
    if (do_db && c16 == 0) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) dbpart[(size_t)blockIdx.x * Cout + co0 + m * 16 + q * 4 + r] = accb[m][r];
    }
}

// dw[co][ci][kh][kw] (+)= sum_chunk slab[chunk][tap][co][ci];  db[co] (+)= sum_chunk dbpart
// block = 64 consecutive slab elements x 4 waves, each wave sums a quarter of the chunks
// (independent loads in flight), fixed-order combine in LDS -> bitwise reproducible.
__global__ __launch_bounds__(256) void k_wgrad_finalize(int nchunk, int Cout, int Cin, int cout_valid,
                                                        const float* __restrict__ part,
                                                        const float* __restrict__ dbpart, float* dw, float* db,
                                                        int accumulate) {
    __shared__ float red[4][64];
    const size_t per = (size_t)9 * Cout * Cin;
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const size_t i = (size_t)blockIdx.x * 64 + lane;
    const int q0 = (nchunk * g) / 4, q1 = (nchunk * (g + 1)) / 4;
    float s = 0.f;
    if (i < per) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int c = q0;
        for (; c + 3 < q1; c += 4) {
            s0 += part[(size_t)c * per + i];
            s1 += part[(size_t)(c + 1) * per + i];
            s2 += part[(size_t)(c + 2) * per + i];
            s3 += part[(size_t)(c + 3) * per + i];
        }
        for (; c < q1; ++c) s0 += part[(size_t)c * per + i];
        s = (s0 + s1) + (s2 + s3);
    }
    red[g][lane] = s;
    __syncthreads();
    if (g == 0 && i < per) {
        const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        const int ci = (int)(i % Cin);
        const int co = (int)((i / Cin) % Cout);
        const int tap = (int)(i / ((size_t)Cin * Cout));
        if (co < cout_valid) {
            float* o = dw + ((size_t)co * Cin + ci) * 9 + tap;
            *o = accumulate ? *o + t : t;
        }
    }
    if (db && blockIdx.x == 0 && g == 1) {
        for (int co = lane; co < cout_valid; co += 64) {
            float t = 0.f;
            for (int c = 0; c < nchunk; ++c) t += dbpart[(size_t)c * Cout + co];
            db[co] = accumulate ? db[co] + t : t;
        }
    }
}

int wgrad_geom(const fen_wgrad_desc* d, int* nchunk, int* tpc, int* cot) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int ntiles = d->B * tpi;
    *cot = d->Cout % 64 == 0 ? 64 : 16;
    const int yz = (d->Cout / *cot) * (d->Cin / 64);
    int t = (ntiles * yz + 255) / 256;  // target ~256 blocks
    if (t < 1) t = 1;
    *tpc = t;
    *nchunk = (ntiles + t - 1) / t;
    return FEN_OK;
}

}  // namespace

extern "C" size_t fen_wgrad_work_floats(const fen_wgrad_desc* d) {
    if (!d || d->B <= 0 || d->Cin <= 0 || d->Cout <= 0) return 0;
    int nchunk, tpc, cot;
    wgrad_geom(d, &nchunk, &tpc, &cot);
    return (size_t)nchunk * 9 * d->Cout * d->Cin + (size_t)nchunk * d->Cout;
}

extern "C" int fen_wgrad3x3(const fen_wgrad_desc* d, void* stream) {
    if (!d || !d->x || !d->dy || !d->dw || !d->work) return FEN_EINVAL;
    if (d->dtype != FEN_F32 && d->dtype != FEN_BF16) return FEN_EINVAL;
    if (d->B <= 0 || d->H <= 0 || d->W <= 0 || d->Cin % 64 || d->Cout % 16 || d->cout_valid <= 0 ||
        d->cout_valid > d->Cout)
        return FEN_EUNSUPPORTED;
    int nchunk, tpc, cot;
    wgrad_geom(d, &nchunk, &tpc, &cot);
    hipStream_t s = (hipStream_t)stream;
    float* part = d->work;
    float* dbpart = d->work + (size_t)nchunk * 9 * d->Cout * d->Cin;
    dim3 grid(nchunk, d->Cout / cot, d->Cin / 64);
    const int npx = d->dtype == FEN_BF16 ? 1 : 2;
    const int npy = d->dtype == FEN_BF16 ? 1 : (cot * 4 > 128 ? 2 : 1);
    const size_t lds = (size_t)npx * PANEL_HALO + (size_t)npy * PANEL_TILE;
    if (d->dtype == FEN_BF16) {
        if (cot == 64) hipLaunchKernelGGL((k_wgrad<bf16, 64>), grid, dim3(576), lds, s, *d, tpc, part, dbpart);
        else hipLaunchKernelGGL((k_wgrad<bf16, 16>), grid, dim3(576), lds, s, *d, tpc, part, dbpart);
    } else {
        if (cot == 64) hipLaunchKernelGGL((k_wgrad<float, 64>), grid, dim3(576), lds, s, *d, tpc, part, dbpart);
        else hipLaunchKernelGGL((k_wgrad<float, 16>), grid, dim3(576), lds, s, *d, tpc, part, dbpart);
    }
    FEN_CHECK_LAUNCH();
    const size_t per = (size_t)9 * d->Cout * d->Cin;
    const int nb = (int)((per + 63) / 64);
    hipLaunchKernelGGL(k_wgrad_finalize, dim3(nb), dim3(256), 0, s, nchunk, d->Cout, d->Cin, d->cout_valid,
                       part, dbpart, d->dw, d->db, d->accumulate);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

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

// the persistent wgrad's operand DMA (x halo, dy tile: read once per job); A/B: WG_LOAD_NT
#ifdef WG_LOAD_NT
#define WG_DMA dma16_nt
#else
#define WG_DMA dma16
#endif

namespace {

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
            // channels past Cin (a partial 64-ci group: Lite's 32 channels) stage as zeros
            if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W &&
                (ci0 + pn * CK) * (int)sizeof(T) + ch * 16 < Cin * (int)sizeof(T))
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
                if (ci < Cin) slab[((size_t)tap * Cout + co) * Cin + ci] = acc[m][n][r];
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


// ------------------------------------------------------------------------------------
// k_wgrad_p: bf16, Cout % 64 == 0, Cin % 64 == 0 -- the network's 64-channel wgrads.
// One 512-thread block per CU walks a contiguous chunk of 16x16-pixel tiles.  Per tile the
// 18x18 input halo (64 ci from ci0) and the 16x16 dy tile (64 co from co0) are streamed by
// LDS-DMA into one of two slots while the MFMAs run on the other.  8 waves = 2 co halves x
// 4 ci quarters; every wave accumulates 32 co x (9 taps x 16 ci) in registers (18 16x16
// accumulators), K = pixels, fragments read with ds_read_b64_tr_b16.  Both LDS images key
// their 16-B chunk positions by bits 1 and 3 of the pixel column (wkey), which makes every
// transposed fragment read bank-conflict free.  The bias gradient rides along as MFMAs
// against a ones fragment, spread over the 4 ci-quarter waves (2 of the 8 k-steps each).
//
// A launch carries up to WG_MAXJ jobs of one shape (fen_wgrad3x3_multi): the grid's x
// blocks are (job, chunk) pairs, so n jobs share the CUs and each block reduces n x as many
// tiles into its one fp32 slab -- the slabs (147 KB per block for a 64x64 conv, written
// and re-read by the finalize) shrink n-fold.  A second launch sums each job's slabs in a
// fixed order (bitwise reproducible) into its OIHW dW / db.
// ------------------------------------------------------------------------------------
constexpr int WG_MAXJ = FEN_WGRAD_MAXJOBS;

// per-job operands (the shape is common to the launch: jobs.d[0])
struct WgJobs {
    const void* x[WG_MAXJ];
    const void* dy[WG_MAXJ];
    int n, nchunk, tpc;
};

__device__ __forceinline__ int wkey(int col) { return (((col >> 1) & 1) << 1) | (((col >> 3) & 1) << 2); }
// COT = 16 (conv_last's zero-padded 16-channel dL/dsr): 32-B dy pixel rows; pixels 8..15 of
// each 16 trade places in groups of 4 so a transposed read's two 8-pixel halves fall in
// different bank halves (an involution: the same map converts LDS <-> tile pixel index)
__device__ __forceinline__ int pswap16(int p) { return p ^ (((p >> 3) & 1) << 2); }

// COT = 64: 8 waves = 2 co halves x 4 ci quarters; COT = 16: 4 waves = 4 ci quarters
template <int COT>
struct WgCfg {
    static constexpr int NW = COT == 64 ? 8 : 4;
    static constexpr int MC = COT == 64 ? 2 : 1;            // 16-row co blocks per wave
    static constexpr int TILE = 256 * COT * 2;              // dy tile image
    static constexpr int TILE_DMA = TILE / 1024;            // 32 / 8 pieces
    static constexpr int SLOT = HALO_SLOT + TILE;           // 2 slots
};

template <int COT>
__global__ __launch_bounds__(512, 1) void k_wgrad_p(const fen_wgrad_desc d, const WgJobs J, float* part) {
    using Cfg = WgCfg<COT>;
    constexpr int NW = Cfg::NW, MC = Cfg::MC;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int ch = COT == 64 ? (wave & 1) : 0, cq = COT == 64 ? (wave >> 1) : wave;
    const int q = lane >> 4, c16 = lane & 15, qq = c16 >> 2, pp = c16 & 3;
    const int H = d.H, W = d.W, Cin = d.Cin, Cout = d.Cout;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int ntiles = d.B * tpi;
    const int co0 = blockIdx.y * COT, ci0 = blockIdx.z * 64;
    // consecutive (job, chunk) slots -- neighbouring tiles of one job, sharing halo rows -- on
    // one XCD; with gridDim.x a multiple of 8 the dispatch XCD is blockIdx.x % 8 whatever y, z
    int slot = blockIdx.x;
    const int gx = (int)gridDim.x;
    if ((gx & 7) == 0) slot = (slot & 7) * (gx >> 3) + (slot >> 3);
    const int job = __builtin_amdgcn_readfirstlane(slot / J.nchunk);
    const int chunk = slot - job * J.nchunk;
    const int t_begin = chunk * J.tpc, t_end = min(t_begin + J.tpc, ntiles);
    const i32x4 xr = make_rsrc(J.x[job], (unsigned)((size_t)d.B * H * W * Cin * 2));
    const i32x4 yr = make_rsrc(J.dy[job], (unsigned)((size_t)d.B * H * W * Cout * 2));

    // every wave issues its share of the tile's 41 halo + TILE_DMA dy pieces: piece k of a
    // wave is i = wave + NW k.  Its lanes' pixel (dr, dc) relative to the tile origin and byte
    // offset from that origin's first channel are fixed for the block, worked out once here
    // (dr = -1000 for the halo's padding lanes: always out of bounds); per tile a piece is a
    // bounds test and an add (the integer divisions per piece and tile were most of the
    // kernel's VALU)
    constexpr int NPC = (HALO_DMA + Cfg::TILE_DMA + NW - 1) / NW;
    int prel[NPC], ppos[NPC];
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
        const int i = wave + NW * k;
        int dr = -1000, dc = 0, rel = 0;
        if (i < HALO_DMA) {
            const int s = i * 64 + lane, p = s >> 3, pos = s & 7;
            const int hr = p / HALO, hc = p - hr * HALO;
            const int c = pos ^ wkey(hc);
            if (s < HP * 8) {
                dr = hr - 1;
                dc = hc - 1;
            }
            rel = ((dr * W + dc) * Cin + c * 8) * 2;
        } else if (i < HALO_DMA + Cfg::TILE_DMA) {
            const int s = (i - HALO_DMA) * 64 + lane;
            int p, c;
            if constexpr (COT == 64) {
                p = s >> 3;
                c = (s & 7) ^ wkey(p & 15);
            } else {
                p = pswap16(s >> 1);
                c = s & 1;
            }
            dr = p >> 4;
            dc = p & 15;
            rel = ((dr * W + dc) * Cout + c * 8) * 2;
        }
        prel[k] = rel;
        ppos[k] = (dr << 16) | (dc & 0xffff);
    }
    auto issue = [&](int t, const char* slotp) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const unsigned hbase = lds_addr(slotp), ybase = lds_addr(slotp + HALO_SLOT);
        const int xb = (((b * H + h0) * W + w0) * Cin + ci0) * 2;
        const int yb = (((b * H + h0) * W + w0) * Cout + co0) * 2;
#pragma unroll
        for (int k = 0; k < NPC; ++k) {
            const int i = wave + NW * k;
            if (i < HALO_DMA + Cfg::TILE_DMA) {
                const int gh = h0 + (ppos[k] >> 16), gw = w0 + ((ppos[k] << 16) >> 16);
                const bool in = (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
                if (i < HALO_DMA)
                    WG_DMA(xr, __builtin_amdgcn_readfirstlane(hbase + i * 1024), in ? xb + prel[k] : 0x7ffffff0);
                else
                    WG_DMA(yr, __builtin_amdgcn_readfirstlane(ybase + (i - HALO_DMA) * 1024),
                          in ? yb + prel[k] : 0x7ffffff0);
            }
        }
    };

    // per-lane fragment offsets (see k_wgrad for the transposed-read lane mapping): lane
    // (q, qq, pp) of half h reads pixel k = 8q + 4h + qq of the 32-pixel k-step, 4 channels
    // from 4*pp.  A (dy): + s * (32 px of the dy image); B (halo, tap kh,kw): + (2s + kh) * 2304.
    constexpr int ASTEP = 32 * COT * 2;
    int offA[2][MC], offB[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int k = 8 * q + 4 * h + qq, r = k >> 4, pc = k & 15;
#pragma unroll
        for (int m = 0; m < MC; ++m) {
            const int c = ch * 32 + m * 16 + 4 * pp;
            if constexpr (COT == 64)
                offA[h][m] = (r * 16 + pc) * 128 + (((c >> 3) ^ wkey(pc)) << 4) + (c & 7) * 2;
            else
                offA[h][m] = pswap16(r * 16 + pc) * 32 + c * 2;
        }
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int c = cq * 16 + 4 * pp, hc = pc + kw;
            offB[h][kw] = (r * HALO + hc) * 128 + (((c >> 3) ^ wkey(hc)) << 4) + (c & 7) * 2;
        }
    }

    f32x4 acc[MC][9], accb[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) {
        accb[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const uint4 ones = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);

    if (t_begin < t_end) issue(t_begin, smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int k = 0, t = t_begin; t < t_end; ++k, ++t) {
        const char* cur = smem + (k & 1) * Cfg::SLOT;
#ifndef WG_NODMA   // diagnostic build: no next-tile loads (times the MFMA/LDS-read body alone)
        if (t + 1 < t_end) issue(t + 1, smem + ((k + 1) & 1) * Cfg::SLOT);
#endif
        const char* hx = cur;
        const char* ty = cur + HALO_SLOT;
        uint4 A0[MC], B0[9], A1[MC], B1[9];
        auto loadA = [&](int s, uint4 (&A)[MC], int h, int m) {
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ty + offA[h][m] + s * ASTEP));
            const uint2 u = __builtin_bit_cast(uint2, v);
            if (h == 0) { A[m].x = u.x; A[m].y = u.y; } else { A[m].z = u.x; A[m].w = u.y; }
        };
        auto loadB = [&](int s, uint4 (&Bf)[9], int h, int tap) {
            const int kh = tap / 3, kw = tap % 3;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4*)(hx + offB[h][kw] + (2 * s + kh) * (HALO * 128)));
            const uint2 u = __builtin_bit_cast(uint2, v);
            if (h == 0) { Bf[tap].x = u.x; Bf[tap].y = u.y; } else { Bf[tap].z = u.x; Bf[tap].w = u.y; }
        };
        // the (MC + 9) x 2 fragment reads of step s, in the order the tap-major MFMAs consume them
        auto load = [&](int s, uint4 (&A)[MC], uint4 (&Bf)[9]) {
#pragma unroll
            for (int m = 0; m < MC; ++m) {
                loadA(s, A, 0, m);
                loadA(s, A, 1, m);
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                loadB(s, Bf, 0, tap);
                loadB(s, Bf, 1, tap);
            }
        };
        auto mma = [&](int s, const uint4 (&A)[MC], const uint4 (&Bf)[9]) {
#ifdef WG_NOMMA     // diagnostic build: no MFMAs (times the loads alone)
            return;
#endif
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int m = 0; m < MC; ++m) mma16<bf16>(acc[m][tap], A[m], Bf[tap]);
            if ((s & 3) == cq) {
#pragma unroll
                for (int m = 0; m < MC; ++m) mma16<bf16>(accb[m], A[m], ones);
            }
        };
        // WG_BURST: the next step's reads as one burst ahead of the MFMAs (A/B); by default
        // they go out between the MFMAs (two per MFMA first, then one), so the two waves of a
        // SIMD, which leave the tile barrier together, do not drain the matrix pipe at once
        auto spread = [&]() {
#ifndef WG_BURST
            constexpr int NR = 2 * (MC + 9), NM = 9 * MC, N2 = NR - NM;   // reads, MFMAs, double slots
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (i < N2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                else __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
#endif
        };
        load(0, A0, B0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 8; s += 2) {
            load(s + 1, A1, B1);
#ifdef WG_BURST
            __builtin_amdgcn_sched_barrier(0);
#endif
            mma(s, A0, B0);
            spread();
            __builtin_amdgcn_sched_barrier(0);
            if (s + 2 < 8) load(s + 2, A0, B0);
#ifdef WG_BURST
            __builtin_amdgcn_sched_barrier(0);
#endif
            mma(s + 1, A1, B1);
            if (s + 2 < 8) spread();
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next tile's pieces landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                         // ... for everyone; cur is free
    }

    // slab layout [tap][Cout][Cin] (+ [Cout] bias): 16 lanes store 64 contiguous bytes; the
    // OIHW order [Cout][Cin][9] put lanes 36 B apart (scattered partial-line writes of all
    // blocks at once at the end of the launch).  k_wgrad_fin transposes on its one write.
    float* slab = part + (size_t)slot * ((size_t)Cout * Cin * 9 + Cout);
#pragma unroll
    for (int m = 0; m < MC; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = co0 + ch * 32 + m * 16 + 4 * q + r, ci = ci0 + cq * 16 + c16;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) slab[((size_t)tap * Cout + co) * Cin + ci] = acc[m][tap][r];
        }
    if (ci0 == 0) {
        float* red = (float*)smem;   // [4 cq][COT co]; no DMA in flight, last barrier passed
        if (c16 == 0) {
#pragma unroll
            for (int m = 0; m < MC; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[cq * COT + ch * 32 + m * 16 + 4 * q + r] = accb[m][r];
        }
        __syncthreads();
        if (tid < COT)
            slab[(size_t)Cout * Cin * 9 + co0 + tid] =
                (red[tid] + red[COT + tid]) + (red[2 * COT + tid] + red[3 * COT + tid]);
    }
}

// per-job outputs of the finalize
struct WgFinJobs {
    float* dw[WG_MAXJ];
    float* db[WG_MAXJ];
    int accumulate[WG_MAXJ];
};

// dw (+)= sum_chunk slab[chunk][tap][co][ci] (co < cout_valid, written OIHW), db (+)= sum_chunk
// slab[chunk][Cout*Cin*9 + co]: a block owns FIN_COLS float4 columns (4 ci of one (tap, co));
// lane = (column, sub-stream), so the block's 8 waves split the chunks into 8 * 64 / FIN_COLS
// streams, combined in a fixed order in LDS (bitwise reproducible).  64 columns per block
// (144 blocks for a 64x64 wgrad): 16 columns (576 blocks, 4x the streams) measured 0.5%
// slower on the training step -- the 37.7 MB slab read runs at ~5 TB/s either way.
// blockIdx.y = job: its slabs are chunks [job * nchunk, (job + 1) * nchunk).
constexpr int FIN_COLS = 64;
__global__ __launch_bounds__(512) void k_wgrad_fin(int nchunk, int stride4, int nw4, int nb, int boff4, int Cout,
                                                   int Cin, const float4* __restrict__ part_all, const WgFinJobs F) {
    constexpr int SUB = 64 / FIN_COLS, NS = 8 * SUB;
    __shared__ float4 red[NS][FIN_COLS];
    const int job = blockIdx.y;
    const float4* part = part_all + (size_t)job * nchunk * stride4;
    float* dw = F.dw[job];
    float* db = F.db[job];
    const int accumulate = F.accumulate[job];
    const int lane = threadIdx.x & 63, w = wave_id();
    const int cl = lane % FIN_COLS, st = w * SUB + lane / FIN_COLS;
    const int j = blockIdx.x * FIN_COLS + cl;
    const int nb4 = (nb + 3) / 4;
    const bool isw = j < nw4, isb = !isw && j < nw4 + nb4;
    const int col = isw ? j : boff4 + (j - nw4);
    const int c0 = (nchunk * st) / NS, c1 = (nchunk * (st + 1)) / NS;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, s3 = s0;
    if (isw || isb) {
        const float4* p = part + col;
        int c = c0;
        for (; c + 3 < c1; c += 4) {
            const float4 a = p[(size_t)c * stride4], b = p[(size_t)(c + 1) * stride4];
            const float4 e = p[(size_t)(c + 2) * stride4], f = p[(size_t)(c + 3) * stride4];
            s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
            s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
            s2.x += e.x; s2.y += e.y; s2.z += e.z; s2.w += e.w;
            s3.x += f.x; s3.y += f.y; s3.z += f.z; s3.w += f.w;
        }
        for (; c < c1; ++c) {
            const float4 a = p[(size_t)c * stride4];
            s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
        }
    }
    red[st][cl] = make_float4((s0.x + s1.x) + (s2.x + s3.x), (s0.y + s1.y) + (s2.y + s3.y),
                              (s0.z + s1.z) + (s2.z + s3.z), (s0.w + s1.w) + (s2.w + s3.w));
    __syncthreads();
    if (w == 0 && lane < FIN_COLS && (isw || isb)) {          // lane == cl here
        float4 t = red[0][cl];
#pragma unroll
        for (int k = 1; k < NS; ++k) {
            const float4 a = red[k][cl];
            t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
        }
        const float v[4] = {t.x, t.y, t.z, t.w};
        if (isw) {
            const int e0 = j * 4, tap = e0 / (Cout * Cin), rem = e0 - tap * (Cout * Cin);
            const int co = rem / Cin, ci = rem - co * Cin;
            if (co < nb) {
                float* o = dw + ((size_t)co * Cin + ci) * 9 + tap;   // scalar stores (OIHW, stride 9)
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e * 9] = accumulate ? o[e * 9] + v[e] : v[e];
            }
        } else if (db) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int co = (j - nw4) * 4 + e;
                if (co < nb) db[co] = accumulate ? db[co] + v[e] : v[e];
            }
        }
    }
}

// the persistent kernel: bf16, Cin % 64 == 0, Cout % 64 == 0 or Cout == 16, 32-bit offsets
bool wgrad_use_p(const fen_wgrad_desc* d) {
    const size_t xb = (size_t)d->B * d->H * d->W * d->Cin * 2, yb = (size_t)d->B * d->H * d->W * d->Cout * 2;
    return d->dtype == FEN_BF16 && (d->Cout % 64 == 0 || d->Cout == 16) && d->Cin % 64 == 0 && xb < 0x7fff0000u &&
           yb < 0x7fff0000u;
}

int wgrad_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            cus = n;
        else
            cus = 256;
    }
    return cus;
}

// tiles per chunk / chunks per job for njobs jobs sharing ~256 blocks
int wgrad_geom(const fen_wgrad_desc* d, int njobs, int* nchunk, int* tpc, int* cot) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int ntiles = d->B * tpi;
    *cot = d->Cout % 64 == 0 ? 64 : 16;
    const int yz = (d->Cout / *cot) * ((d->Cin + 63) / 64);
    int t = (ntiles * yz * njobs + 255) / 256;  // target ~256 blocks
    if (t < 1) t = 1;
    // ... and never more: one block per CU, so a 257th block is a second wave of a whole chunk
    // (5 jobs of 512 tiles at t = 10 would be 5 x 52 = 260 blocks; t = 11 gives 235)
    // Bounded: once t >= ntiles a job is one chunk, and njobs * yz > 256 simply runs more than
    // one wave of blocks (the persistent form still sums each chunk into its own slab).
    while (t < ntiles && njobs * yz * ((ntiles + t - 1) / t) > 256) ++t;
    *tpc = t;
    *nchunk = (ntiles + t - 1) / t;
    return FEN_OK;
}

size_t slab_floats(const fen_wgrad_desc* d) { return (size_t)d->Cout * d->Cin * 9 + d->Cout; }

bool same_shape(const fen_wgrad_desc* a, const fen_wgrad_desc* b) {
    return a->dtype == b->dtype && a->B == b->B && a->H == b->H && a->W == b->W && a->Cin == b->Cin &&
           a->Cout == b->Cout && a->cout_valid == b->cout_valid;
}

int check_desc(const fen_wgrad_desc* d) {
    if (!d || !d->x || !d->dy || !d->dw) return FEN_EINVAL;
    if (d->dtype != FEN_F32 && d->dtype != FEN_BF16) return FEN_EINVAL;
    // Cin: 16-B channel chunks (% 8 bf16, % 4 f32); a partial last 64-ci group reads zeros
    if (d->B <= 0 || d->H <= 0 || d->W <= 0 || (d->Cin * (d->dtype == FEN_F32 ? 4 : 2)) % 16 || d->Cout % 16 ||
        d->cout_valid <= 0 || d->cout_valid > d->Cout)
        return FEN_EUNSUPPORTED;
    return FEN_OK;
}

// n jobs of one persistent-kernel shape, workspace `work`
int launch_p(int n, const fen_wgrad_desc* ds, float* work, hipStream_t s) {
    const fen_wgrad_desc* d = &ds[0];
    int nchunk, tpc, cot;
    wgrad_geom(d, n, &nchunk, &tpc, &cot);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_wgrad_p<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * WgCfg<64>::SLOT);
        (void)hipFuncSetAttribute((const void*)k_wgrad_p<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * WgCfg<16>::SLOT);
        attr = true;
    }
    WgJobs J{};
    WgFinJobs F{};
    for (int i = 0; i < n; ++i) {
        J.x[i] = ds[i].x;
        J.dy[i] = ds[i].dy;
        F.dw[i] = ds[i].dw;
        F.db[i] = ds[i].db;
        F.accumulate[i] = ds[i].accumulate;
    }
    J.n = n;
    J.nchunk = nchunk;
    J.tpc = tpc;
    if (cot == 64)
        hipLaunchKernelGGL(k_wgrad_p<64>, dim3(n * nchunk, d->Cout / 64, d->Cin / 64), dim3(64 * WgCfg<64>::NW),
                           2 * WgCfg<64>::SLOT, s, *d, J, work);
    else
        hipLaunchKernelGGL(k_wgrad_p<16>, dim3(n * nchunk, 1, d->Cin / 64), dim3(64 * WgCfg<16>::NW),
                           2 * WgCfg<16>::SLOT, s, *d, J, work);
    FEN_CHECK_LAUNCH();
    const int stride4 = (int)(slab_floats(d) / 4);
    const int nw4 = d->Cout * d->Cin * 9 / 4;   // tap-major: rows co >= cout_valid skipped
    const int boff4 = d->Cout * d->Cin * 9 / 4;
    const int ncol = nw4 + (d->cout_valid + 3) / 4;
    hipLaunchKernelGGL(k_wgrad_fin, dim3((ncol + FIN_COLS - 1) / FIN_COLS, n), dim3(512), 0, s, nchunk, stride4, nw4,
                       d->cout_valid, boff4, d->Cout, d->Cin, (const float4*)work, F);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

}  // namespace

extern "C" size_t fen_wgrad_work_floats(const fen_wgrad_desc* d) {
    if (!d || d->B <= 0 || d->Cin <= 0 || d->Cout <= 0) return 0;
    int nchunk, tpc, cot;
    wgrad_geom(d, 1, &nchunk, &tpc, &cot);
    if (wgrad_use_p(d)) return (size_t)nchunk * slab_floats(d);
    return (size_t)nchunk * 9 * d->Cout * d->Cin + (size_t)nchunk * d->Cout;
}

extern "C" size_t fen_wgrad_multi_work_floats(int n, const fen_wgrad_desc* ds) {
    if (!ds || n <= 0 || n > WG_MAXJ) return 0;
    const size_t one = fen_wgrad_work_floats(&ds[0]);
    if (!wgrad_use_p(&ds[0])) return one;   // jobs run one after another in the one workspace
    int nchunk, tpc, cot;
    wgrad_geom(&ds[0], n, &nchunk, &tpc, &cot);
    const size_t multi = (size_t)n * nchunk * slab_floats(&ds[0]);
    return multi > one ? multi : one;
}

extern "C" int fen_wgrad3x3(const fen_wgrad_desc* d, void* stream) {
    const int st = check_desc(d);
    if (st != FEN_OK) return st;
    if (!d->work) return FEN_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (wgrad_use_p(d)) return launch_p(1, d, d->work, s);
    int nchunk, tpc, cot;
    wgrad_geom(d, 1, &nchunk, &tpc, &cot);
    float* part = d->work;
    float* dbpart = d->work + (size_t)nchunk * 9 * d->Cout * d->Cin;
    dim3 grid(nchunk, d->Cout / cot, (d->Cin + 63) / 64);
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

extern "C" int fen_wgrad3x3_multi(int n, const fen_wgrad_desc* ds, void* stream) {
    if (!ds || n <= 0 || n > WG_MAXJ || !ds[0].work) return FEN_EINVAL;
    for (int i = 0; i < n; ++i) {
        const int st = check_desc(&ds[i]);
        if (st != FEN_OK) return st;
        if (!same_shape(&ds[0], &ds[i])) return FEN_EINVAL;
    }
    hipStream_t s = (hipStream_t)stream;
    if (wgrad_use_p(&ds[0])) return launch_p(n, ds, ds[0].work, s);
    for (int i = 0; i < n; ++i) {   // generic kernel: one job at a time in the shared workspace
        fen_wgrad_desc d = ds[i];
        d.work = ds[0].work;
        const int st = fen_wgrad3x3(&d, stream);
        if (st != FEN_OK) return st;
    }
    return FEN_OK;
}

// 3x3 / stride 1 / pad 1 convolution on NHWC activations as an implicit GEMM on MFMA (gfx950).
//
// Replaces every nn.Conv2d(k=3, pad=1) forward of the hot path (reference blocks.py:123-131,
// 182-183, 211-214; custom.py:109-112, 121-124) and, given flipped/transposed weights
// (fen_pack_conv_w mode 2), the data-gradient of each of them.
//
// Output tile = 16x16 pixels x COT output channels, 4 waves; each wave owns 4 output rows:
//   D[co][px] = sum_k W[co][k] * X[k][px],  k = (tap, ci):  A = weights, B = pixels,
//   MT*4 accumulators of v_mfma_f32_16x16x32_{bf16,f16} (or 4x v_mfma_f32_16x16x4_f32 per 16 B).
// Every LDS image has 128-B rows (64 bf16/fp16 / 32 f32 channels = one "panel") with the
// 16-B chunks XOR-swizzled by (row>>1)&7 -> conflict-free ds_read_b128 fragment reads.
//
// Two kernels:
//  * k_conv3x3_p (bf16 / fp16, Cin == 64 -- every 64-channel conv of the network, forward and
//    dgrad, the x2 upsampler and conv_last): PERSISTENT, one 256-thread block per CU.
//    The block's whole filter (9 taps x COT x 64, 72 KB) stays resident in LDS; the
//    18x18-pixel input halo of the next tile is streamed by LDS-DMA (buffer_load ... lds,
//    zero padding via the buffer range check) into a second buffer while the MFMAs run
//    on the current one: one barrier per tile, none per tap.  156.7 KB LDS.
//  * k_conv3x3_s (any Cin multiple of 16 B, bf16 / fp16 and f32): weights streamed per tap
//    through a double-buffered LDS tile, halo staged through registers; 2 blocks per CU.
//    Used for f32 (the parity path), for Cin > 64 (upsampler dgrad, 128-ch variant) and for
//    Cin < 64 (FaceEnhanceNetLite's 32 channels; the panel's upper half is zeros).
// The epilogue fuses bias, residual adds, PReLU (fwd) or PReLU-backward (dgrad),
// PixelShuffle / inverse-PixelShuffle stores, SE global-average-pool partials, and for
// conv_last the bicubic skip + eval clamp + L1-loss gradient.
#include "fen_common.h"

#include <type_traits>

extern "C" int fen_maxpool2(int dtype, int B, int H, int W, int C, const void* x, void* y, void* stream);   // vgg.hip

namespace {

// Diagnostic build only (-DFEN_STAMPS, tools/stamp_conv.py): per-block s_memrealtime /
// s_memtime stamps of the persistent kernel's phases into d.loss_part (unused by the
// forward epilogues), [block][wave][16 stamps][realtime, memtime] u64.  In the real build no stamp executes.
#ifdef FEN_STAMPS
#define FEN_STAMP(i)                                                                          \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long _rt, _mt;                                                          \
        asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"                 \
                     : "=s"(_rt), "=s"(_mt)::"memory");                                       \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        if (d.loss_part && (threadIdx.x & 63) == 0 && (i) < 16) {    /* never through NULL */    \
            unsigned long long* _p =                                                          \
                (unsigned long long*)d.loss_part + ((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 32; \
            _p[2 * (i)] = _rt;                                                                \
            _p[2 * (i) + 1] = _mt;                                                            \
        }                                                                                     \
    } while (0)
#else
#define FEN_STAMP(i) \
    do {             \
    } while (0)
#endif

// The conv kernels keep the wave id as tid >> 6 (divergent to hipcc, so their per-wave roles
// compile to exec-masked code): the readfirstlane form (wave_id(), fen_common.h) measured
// slower here -- upsampler 188.9 -> 195.7 us, dgrads +0.8 / +1.2 us (tools/gpu_t10.sh) --
// while it sped up k_rcab and k_conv_last.

// s_waitcnt vmcnt(n) for a runtime n (the immediate must be a literal): waits until at
// most n of this wave's vector-memory ops are outstanding.  Ops retire in issue order, so
// with n = number of stores issued after the halo prefetch, the prefetch has landed while
// the tile's output stores keep draining behind the next tile's MFMAs.
__device__ __forceinline__ void wait_vm_upto(int n) {
    switch (n) {
#define FEN_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        FEN_VMC(1) FEN_VMC(2) FEN_VMC(3) FEN_VMC(4) FEN_VMC(5) FEN_VMC(6) FEN_VMC(7) FEN_VMC(8)
        FEN_VMC(9) FEN_VMC(10) FEN_VMC(11) FEN_VMC(12) FEN_VMC(13) FEN_VMC(14) FEN_VMC(15) FEN_VMC(16)
        FEN_VMC(17) FEN_VMC(18) FEN_VMC(19) FEN_VMC(20) FEN_VMC(21) FEN_VMC(22) FEN_VMC(23) FEN_VMC(24)
        FEN_VMC(25) FEN_VMC(26) FEN_VMC(27) FEN_VMC(28) FEN_VMC(29) FEN_VMC(30) FEN_VMC(31) FEN_VMC(32)
#undef FEN_VMC
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// Output store instructions a wave is guaranteed to issue in conv_epilogue after the halo
// prefetch (full interior tiles, plain/SHUFFLE stores); 0 = "wait for everything".
__device__ __forceinline__ int epi_store_count(const fen_conv_desc& d, int h0, int w0, int mtnt) {
    if ((d.epi & (FEN_EPI_LAST | FEN_EPI_UNSHUFFLE)) || h0 + 16 > d.H || w0 + 16 > d.W) return 0;
    return mtnt * (((d.epi & FEN_EPI_PRELU) && d.y_pre) ? 2 : 1);
}

// Per-channel epilogue constants of one wave's output channels, loaded once per block
// (bias[co] and the PReLU slope; for SHUFFLE the packed row cp maps to co = 4(cp%Cq)+cp/Cq
// and the slope index to cp%Cq).
template <int MT>
struct EpiConst {
    float bias[MT][4];
    float alpha[MT][4];
};
template <int MT>
__device__ __forceinline__ EpiConst<MT> epi_consts(const fen_conv_desc& d, int cob0) {
    EpiConst<MT> e;
    const int Cout = d.Cout, Cq = Cout >> 2;
    const bool shuf = d.epi & FEN_EPI_SHUFFLE;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cp = cob0 + m * 16 + r;
            const bool ok = cp < Cout;
            const int co = shuf ? 4 * (cp % Cq) + cp / Cq : cp;
            e.bias[m][r] = (ok && (d.epi & FEN_EPI_BIAS)) ? d.bias[co] : 0.f;
            e.alpha[m][r] = (ok && (d.epi & (FEN_EPI_PRELU | FEN_EPI_PRELU_BWD))) ? d.alpha[shuf ? cp % Cq : cp] : 0.f;
        }
    return e;
}

// fen_conv_desc.y_pool: the 2x2 max pool fused into the store (compile-time key bit of the
// persistent kernels' epilogue instantiations; VGG19's conv -> ReLU -> 'M', perceptual.py:50-53).
constexpr int EPIC_MPOOL = 1 << 13;
// A wave's tile piece: rows h0w + n (n < 4, h0w even) x columns w0 + c16 x channels cob0 + m*16
// + 4q + r; o(m, n, r) = the stored activation.  Rows pool inside a lane, columns across lanes
// c16 ^ 1 (DPP): the even lane of a pair keeps pooled row 0 and sends row 1, the odd lane the
// reverse, so every lane stores one pooled pixel's 4 channels.  max commutes with the monotone
// rounding to T, so this equals pooling the stored y (k_maxpool2).
template <typename T, int MT, typename F>
__device__ __forceinline__ void pool2_store(const fen_conv_desc& d, int b, int h0w, int w0, int cob0, int c16,
                                            bool full, F&& o) {
    const int H = d.H, W = d.W, Cout = d.Cout, Hp = H >> 1, Wp = W >> 1;
    const bool odd = c16 & 1;
    const int hp = (h0w >> 1) + (odd ? 1 : 0), wp = (w0 + c16) >> 1;
    const bool ok = full || (2 * hp < H && 2 * wp < W);
    char* base = (char*)d.y_pool + ((((size_t)b * Hp + hp) * Wp + wp) * Cout + cob0) * sizeof(T);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        float res[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float a0 = fmaxf(o(m, 0, r), o(m, 1, r)), a1 = fmaxf(o(m, 2, r), o(m, 3, r));
            const float recv = dpp_f<0xB1>(odd ? a0 : a1);
            res[r] = fmaxf(odd ? a1 : a0, recv);
        }
        if (ok && cob0 + m * 16 < Cout) st4<T>(base + m * 16 * sizeof(T), res);
    }
}

// ------------------------------------------------------------------------------------
// epilogue (shared by both kernels).  acc[m][n][r] = D[co = co0 + m*16 + 4q + r][pixel
// (h0 + wave*4 + n, w0 + c16)].  `stage` (>= 32 KB LDS) enables the 16-bit LDS-staged
// store path (COT == 64 only); `red` is >= 4*COT floats of LDS.  Contains barriers:
// every thread of the block must call it.
// ------------------------------------------------------------------------------------
// Block barrier for LDS hand-offs only.  RAW (persistent kernel): lgkmcnt(0) + s_barrier,
// no memory fence -- a __syncthreads() would also drain the next tile's in-flight halo
// LDS-DMA (vmcnt(0)).  Returns the global store instructions this wave issued in its final
// store phase when the tile is full and every lane stored in each of them (the caller then
// waits vmcnt(that) for the older halo DMA), else 0 (= wait for everything).
template <bool RAW>
__device__ __forceinline__ void epi_barrier() {
    if constexpr (RAW) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    } else {
        __syncthreads();
    }
}

template <typename T, int COT, int WR, int WC, int EPIC = -1, bool RAW = false>
__device__ __forceinline__ int conv_epilogue(const fen_conv_desc& d, f32x4 (&acc)[COT / 16 / WC][16 / WR], int b,
                                             int tlin, int h0, int w0, int co0, char* stage, float* red,
                                             const EpiConst<COT / 16 / WC>& ec) {
    constexpr int MT = COT / 16 / WC, NT = 16 / WR, CW = COT / WC;
    constexpr int NTHR = 64 * WR * WC;
    // EPIC >= 0: the epilogue mode is a compile-time constant (flags | residual count << 8),
    // so every branch on it folds away; -1: read it from the descriptor.
    constexpr bool CT = EPIC >= 0;
    constexpr int NRES = CT ? ((EPIC >> 8) & 3) : 3;
    constexpr bool MPOOL = CT && (EPIC & EPIC_MPOOL);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave % WR, wc = wave / WR;
    const int q = lane >> 4, c16 = lane & 15;
    const int H = d.H, W = d.W, Cout = d.Cout;
    const int epi = CT ? (EPIC & ~(0x300 | EPIC_MPOOL)) : d.epi;
    const int w_ = w0 + c16;
    const bool full = h0 + 16 <= H && w0 + 16 <= W;

    if (epi & FEN_EPI_LAST) {
        // conv_last: rows co = 4q + r; only co < Cout (3) are real.  One bicubic sample per
        // lane: lane (q, c16) computes channel q of pixel c16, then lanes of q == 0 gather.
        const int Hs = H / d.scale, Ws = W / d.scale;
        const float inv = 1.0f / (float)d.scale;
        float lsum = 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int h = h0 + wr * NT + n;
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
                    float v = acc[0][n][r] + ec.bias[0][r] + bq[r];
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
            __syncthreads();
            if (lane == 0) red[wave] = lsum;
            __syncthreads();
            if (tid == 0) {
                float t = 0.f;
                for (int w = 0; w < WR * WC; ++w) t += red[w];
                d.loss_part[tlin] = t;
            }
        }
        return 0;
    }

    const bool shuf = epi & FEN_EPI_SHUFFLE;
    const bool unshuf = epi & FEN_EPI_UNSHUFFLE;
    const int Cq = Cout >> 2;
    float psum[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) psum[m][r] = 0.f;

    bool rec4[MT];                                        // PRELU_BWD from post_in (see fen.h)
#pragma unroll
    for (int m = 0; m < MT; ++m) rec4[m] = (epi & FEN_EPI_PRELU_BWD) && d.post_in && all_pos4(ec.alpha[m]);
    // the PRELU_BWD / DOT operands of the whole tile issued together, branch-free (an invalid
    // pixel re-reads offset 0 and is not used), before pass 1 consumes any: one memory round
    // trip per tile instead of one per (m, n) -- a load under the per-pixel branch with its use
    // right behind it waited for each in turn
    typedef typename std::conditional<sizeof(T) == 2, uint2, uint4>::type RawV;
#ifndef EPI_NOPF
    const bool pin = epi & (FEN_EPI_PRELU_BWD | FEN_EPI_DOT | FEN_EPI_RELU_BWD);
#else   // A/B only: the operands loaded per fragment in pass 1
    const bool pin = false;
#endif
    RawV pvr[MT][NT];
    if (pin) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int cob = co0 + wc * CW + m * 16 + q * 4;
            const char* src = (const char*)(((epi & FEN_EPI_PRELU_BWD) && rec4[m]) ? d.post_in : d.pre_in);
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int h = h0 + wr * NT + n;
                const bool valid = (full || (h < H && w_ < W)) && cob < Cout;
                const size_t oi = valid ? ((size_t)(b * H + h) * W + w_) * Cout + cob : 0;
                pvr[m][n] = *(const RawV*)(src + oi * sizeof(T));
            }
        }
    }
    // pass 1: elementwise epilogue in registers (acc <- pre-activation value)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int cob = co0 + wc * CW + m * 16 + q * 4;      // first of 4 consecutive (packed) channels
        const float* bias4 = ec.bias[m];
        const float* al4 = ec.alpha[m];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int h = h0 + wr * NT + n;
            const bool valid = (full || (h < H && w_ < W)) && cob < Cout;
            const size_t oi = ((size_t)(b * H + h) * W + w_) * Cout + cob;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[m][n][r] + bias4[r];
            if (valid) {
#pragma unroll
                for (int k = 0; k < NRES; ++k) {
                    if (CT || d.res[k]) {
                        float rv[4];
                        ld4<T>((const char*)d.res[k] + oi * sizeof(T), rv);
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += rv[r];
                    }
                }
                if (epi & FEN_EPI_PRELU_BWD) {
                    // post_in (every slope of the group > 0): the PReLU output has the
                    // pre-activation's sign; the slope partials are rescaled by 1 / alpha below
                    float pv[4];
#ifndef EPI_NOPF
                    ld4<T>(&pvr[m][n], pv);
#else
                    ld4<T>((const char*)(rec4[m] ? d.post_in : d.pre_in) + oi * sizeof(T), pv);
#endif
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        psum[m][r] += prelu_dalpha_f(v[r], pv[r]);
                        v[r] = prelu_bwd_f(v[r], pv[r], al4[r]);
                    }
                }
                if (epi & FEN_EPI_RELU_BWD) {
                    float pv[4];
#ifndef EPI_NOPF
                    ld4<T>(&pvr[m][n], pv);
#else
                    ld4<T>((const char*)d.pre_in + oi * sizeof(T), pv);
#endif
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = pv[r] > 0.f ? v[r] : 0.f;
                }
                if (epi & FEN_EPI_DOT) {
                    float pv[4];
#ifndef EPI_NOPF
                    ld4<T>(&pvr[m][n], pv);
#else
                    ld4<T>((const char*)d.pre_in + oi * sizeof(T), pv);
#endif
#pragma unroll
                    for (int r = 0; r < 4; ++r) psum[m][r] += rnd16<T>(v[r]) * pv[r];
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
    if (epi & (FEN_EPI_POOL | FEN_EPI_PRELU_BWD | FEN_EPI_DOT)) {
        // red[] was last read before the previous tile's closing barrier: no barrier needed here
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float s = group16_sum(psum[m][r]) * (rec4[m] ? __builtin_amdgcn_rcpf(ec.alpha[m][r]) : 1.f);
                if (c16 == 0) red[wr * COT + wc * CW + m * 16 + q * 4 + r] = s;
            }
        epi_barrier<RAW>();
        if (tid < COT && co0 + tid < Cout) {
            float t = 0.f;
#pragma unroll
            for (int w = 0; w < WR; ++w) t += red[w * COT + tid];
            d.part[(size_t)tlin * Cout + co0 + tid] = t;
        }
    }

    const bool prelu = epi & FEN_EPI_PRELU;
    auto final_v = [&](float v, int m, int r, int k) -> float {   // value stored for output k (0: y_pre, 1: y)
        if (k == 1 && prelu) return prelu_f(v, ec.alpha[m][r]);
        return v;
    };

    if (stage != nullptr) {
        if constexpr (sizeof(T) == 2 && COT == 64) {
            // ---- 16-bit: stage the 256 x 64 tile in LDS, leave as full 128-B rows ----
            int nst = 0;
            for (int k = 0; k < 2; ++k) {
                void* dst = k == 0 ? d.y_pre : d.y;
                if (k == 0 && (!prelu || !dst)) continue;
                epi_barrier<RAW>();   // every wave is done with the stage (its MFMAs / last reads)
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const int cl = wc * CW + m * 16 + q * 4;
#pragma unroll
                    for (int n = 0; n < NT; ++n) {
                        const int px = (wr * NT + n) * 16 + c16;
                        float v[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = final_v(acc[m][n][r], m, r, k);
                        st4<T>(stage + swz(px, cl >> 3) + (q & 1) * 8, v);
                    }
                }
                epi_barrier<RAW>();
                if (!unshuf) {
                    nst += 256 * 8 / NTHR;
                    for (int i = tid; i < 256 * 8; i += NTHR) {
                        const int px = i >> 3, ch = i & 7;
                        const int h = h0 + (px >> 4), w = w0 + (px & 15);
                        if (h >= H || w >= W) continue;
                        const uint4 v = *(const uint4*)(stage + swz(px, ch));
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
                    nst += 64 * 32 / NTHR;
                    for (int i = tid; i < 64 * 32; i += NTHR) {
                        const int dp = i >> 5, kq = i & 31;
                        const int hh = dp >> 3, ww = dp & 7;
                        const int gh = (h0 >> 1) + hh, gw = (w0 >> 1) + ww;
                        if (gh >= Hh || gw >= Wh) continue;
                        unsigned short e[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int cl = 2 * kq + (j >> 2), t = j & 3;
                            const int px = (2 * hh + (t >> 1)) * 16 + 2 * ww + (t & 1);
                            e[j] = *(const unsigned short*)(stage + swz(px, cl >> 3) + (cl & 7) * 2);
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
            return full ? nst : 0;
        }
    }
    // ---- direct stores from registers ----
    int nst = 0;
    for (int k = 0; k < 2; ++k) {
        void* dst = k == 0 ? d.y_pre : d.y;
        if (k == 0 && (!prelu || !dst)) continue;
        if (MPOOL && d.y_images > 0 && b >= d.y_images) continue;   // (block-uniform)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int cob = co0 + wc * CW + m * 16 + q * 4;
            if (cob >= Cout) continue;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int h = h0 + wr * NT + n;
                if (!full && (h >= H || w_ >= W)) continue;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = final_v(acc[m][n][r], m, r, k);
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
                ++nst;
            }
        }
    }
    if constexpr (MPOOL) {
        static_assert(NT == 4, "pool2_store: 4 rows per wave");
        pool2_store<T, MT>(d, b, h0 + wr * NT, w0, co0 + wc * CW + q * 4, c16, full,
                           [&](int m, int n, int r) { return final_v(acc[m][n][r], m, r, 1); });
    }
    return (full && !unshuf && co0 + COT <= Cout) ? nst : 0;
}

// MFMAs of one tap from a weight tile wt ([COT rows][128 B]) and a halo image
// wave (wr, wc) reads weight rows wc*MT*16 + m*16 + c16 and halo rows wr*NT + n + kh
template <typename T, int MT, int NT>
__device__ __forceinline__ void conv_tap(f32x4 (&acc)[MT][NT], const char* wt, const char* halo, int tap, int wr,
                                         int wc, int q, int c16) {
    const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + q;
        uint4 A[MT], Bf[NT];
#pragma unroll
        for (int m = 0; m < MT; ++m) A[m] = *(const uint4*)(wt + swz(wc * MT * 16 + m * 16 + c16, chunk));
        const char* hb = halo + hcol(c16 + kw, chunk);
#pragma unroll
        for (int n = 0; n < NT; ++n) Bf[n] = *(const uint4*)(hb + (wr * NT + n + kh) * (HALO * 128));
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) mma16<T>(acc[m][n], A[m], Bf[n]);
    }
}

// All 9 taps x 2 k-halves of one tile from an LDS-resident filter, software-pipelined:
// the fragments of step s+1 are read while the MFMAs of step s run (two register sets).
// per_tap(tap) runs once per tap between the MFMA groups (the next tile's halo DMA).
template <typename T, int COT, int MT, int NT, typename F>
__device__ __forceinline__ void conv_tile_resident(f32x4 (&acc)[MT][NT], const char* wts, const char* halo, int wr,
                                                   int wc, int q, int c16, F&& per_tap) {
    uint4 A0[MT], B0[NT], A1[MT], B1[NT];
    const int arow = wc * MT * 16 + c16;
    auto load = [&](int tap, int kk, uint4 (&A)[MT], uint4 (&Bf)[NT]) {
        const int kh = tap / 3, kw = tap - kh * 3;
        const int chunk = kk * 4 + q;
        const char* wt = wts + tap * COT * 128;
#pragma unroll
        for (int m = 0; m < MT; ++m) A[m] = *(const uint4*)(wt + swz(arow + m * 16, chunk));
        const char* hb = halo + hcol(c16 + kw, chunk) + (wr * NT + kh) * (HALO * 128);
#pragma unroll
        for (int n = 0; n < NT; ++n) Bf[n] = *(const uint4*)(hb + n * (HALO * 128));
    };
    auto mma = [&](const uint4 (&A)[MT], const uint4 (&Bf)[NT]) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) mma16<T>(acc[m][n], A[m], Bf[n]);
    };
    // sched_barriers pin the order: each fragment set is read one MFMA group ahead of its use
    load(0, 0, A0, B0);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
        load(tap, 1, A1, B1);
        per_tap(tap);
        __builtin_amdgcn_sched_barrier(0);
        mma(A0, B0);
        __builtin_amdgcn_sched_barrier(0);
        // unconditional (the last tap re-reads tap 0, unused): a conditional load here makes
        // the waitcnt pass merge both paths and drain the prefetch before the next MFMAs
        load(tap == 8 ? 0 : tap + 1, 0, A0, B0);
        __builtin_amdgcn_sched_barrier(0);
        mma(A1, B1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Same tile, halo-row reuse order: for each (kw, k-half) the wave reads its NT+2 halo rows
// once and applies them to all three kh taps (output row n uses halo row n + kh), so one
// group = NT+2 pixel fragments + 3*MT filter fragments for 3*MT*NT MFMAs -- 0.5 LDS reads
// per MFMA at MT=2, NT=4 (tap order: 0.75).  Double-buffered one group ahead.
template <typename T, int COT, int MT, int NT>
__device__ __forceinline__ void conv_tile_rows(f32x4 (&acc)[MT][NT], const char* wts, const char* halo, int wr,
                                               int wc, int q, int c16) {
    constexpr int NB = NT + 2;
    uint4 A0[3][MT], B0[NB], A1[3][MT], B1[NB];
    const int arow = wc * MT * 16 + c16;
    auto load = [&](int g, uint4 (&A)[3][MT], uint4 (&Bf)[NB]) {
        const int kw = g >> 1, kk = g & 1;
        const int chunk = kk * 4 + q;
        const char* hb = halo + hcol(c16 + kw, chunk) + (wr * NT) * (HALO * 128);
#pragma unroll
        for (int n = 0; n < NB; ++n) Bf[n] = *(const uint4*)(hb + n * (HALO * 128));
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const char* wt = wts + (kh * 3 + kw) * COT * 128;
#pragma unroll
            for (int m = 0; m < MT; ++m) A[kh][m] = *(const uint4*)(wt + swz(arow + m * 16, chunk));
        }
    };
    auto mma = [&](const uint4 (&A)[3][MT], const uint4 (&Bf)[NB]) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n) mma16<T>(acc[m][n], A[kh][m], Bf[n + kh]);
    };
    load(0, A0, B0);
#pragma unroll
    for (int g = 0; g < 6; g += 2) {
        load(g + 1, A1, B1);
        __builtin_amdgcn_sched_barrier(0);
        mma(A0, B0);
        __builtin_amdgcn_sched_barrier(0);
        if (g + 2 < 6) load(g + 2, A0, B0);
        __builtin_amdgcn_sched_barrier(0);
        mma(A1, B1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The halo-row-reuse order at lower register cost: 18 steps (kw, k-half, kh); the filter
// fragments of step s+1 and the halo rows of the next (kw, k-half) group are read while
// step s's MFMAs run -- 2*MT + 2*(NT+2) fragment registers (64 at MT=NT=4) instead of
// 6*MT + 2*(NT+2).
template <typename T, int COT, int MT, int NT>
__device__ __forceinline__ void conv_tile_rows2(f32x4 (&acc)[MT][NT], const char* wts, const char* halo, int wr,
                                                int wc, int q, int c16) {
    constexpr int NB = NT + 2;
    uint4 A0[MT], A1[MT], B0[NB], B1[NB];
    const int arow = wc * MT * 16 + c16;
    auto loadB = [&](int g, uint4 (&Bf)[NB]) {
        const int kw = g >> 1, kk = g & 1;
        const char* hb = halo + hcol(c16 + kw, kk * 4 + q) + (wr * NT) * (HALO * 128);
#pragma unroll
        for (int n = 0; n < NB; ++n) Bf[n] = *(const uint4*)(hb + n * (HALO * 128));
    };
    auto loadA = [&](int st, uint4 (&A)[MT]) {
        const int g = st / 3, kh = st % 3, kw = g >> 1, kk = g & 1;
        const char* wt = wts + (kh * 3 + kw) * COT * 128;
#pragma unroll
        for (int m = 0; m < MT; ++m) A[m] = *(const uint4*)(wt + swz(arow + m * 16, kk * 4 + q));
    };
    auto mma = [&](const uint4 (&A)[MT], const uint4 (&Bf)[NB], int kh) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) mma16<T>(acc[m][n], A[m], Bf[n + kh]);
    };
    loadB(0, B0);
    loadA(0, A0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < 6; ++g) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int st = g * 3 + kh;
            int nl = 0;
            if (st + 1 < 18) {
                if (st & 1) loadA(st + 1, A0); else loadA(st + 1, A1);
                nl += MT;
            }
            if (kh == 0 && g + 1 < 6) {
                if (g & 1) loadB(g + 1, B0); else loadB(g + 1, B1);
                nl += NB;
            }
#ifdef G_BURST
            __builtin_amdgcn_sched_barrier(0);
#endif
            if (st & 1) {
                if (g & 1) mma(A1, B1, kh); else mma(A1, B0, kh);
            } else {
                if (g & 1) mma(A0, B1, kh); else mma(A0, B0, kh);
            }
#ifndef G_BURST
            // one wave per SIMD computes while the other group services: the next step's
            // fragment reads go out one per MFMA instead of as a burst ahead of them, so the
            // matrix pipe does not drain while the wave issues them
            if (nl > 0) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
#pragma unroll
            for (int i = 0; i < MT * NT; ++i) {
                if (i < nl) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                if (i + (nl > 0 ? 1 : 0) < MT * NT) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// ------------------------------------------------------------------------------------
// k_conv3x3_p: persistent, resident weights, LDS-DMA double-buffered halo (16-bit, Cin=64)
// ------------------------------------------------------------------------------------
template <typename T, int COT, int WR, int WC, int EPIC>
__global__ __launch_bounds__(64 * WR * WC, 1) void k_conv3x3_p(const fen_conv_desc d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int MT = COT / 16 / WC, NT = 16 / WR, NW = WR * WC;
    constexpr int WBYTES = 9 * COT * 128;
    char* wts = smem;
    char* hbuf = smem + WBYTES;                              // 2 x HALO_SLOT
    float* red = (float*)(smem + WBYTES + 2 * HALO_SLOT);    // WR * COT floats

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave % WR, wc = wave / WR;
    const int q = lane >> 4, c16 = lane & 15;
    const int H = d.H, W = d.W, Cout = d.Cout;
    const int coutp = (Cout + 15) & ~15;
    const int ncot = coutp / COT;
    const int bid = xcd_block();                             // a tile's co blocks + neighbours: one XCD
    const int cot = bid % ncot, co0 = cot * COT;
    const int nslot = gridDim.x / ncot, slot = bid / ncot;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int ntiles = d.B * tpi;

    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)d.w, (short)0, (int)((size_t)9 * coutp * 128), 0x00020000);

    // resident filter: rows r = tap*COT + co_l; lane-linear LDS slots, swizzle on the source
    for (int i = wave; i < WBYTES / 1024; i += NW) {
        const int s = i * 64 + lane;
        const int r = s >> 3, pc = s & 7;
        const int c = pc ^ ((r >> 1) & 7);
        const int tap = r / COT, col = r - tap * COT;
        const int voff = ((tap * coutp + co0 + col) * 64 + c * 8) * 2;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void*)(wts + i * 1024), 16, voff, 0, 0, 0);
    }
    const i32x4 xr4 = make_rsrc(d.x, (unsigned)((size_t)d.B * H * W * 128));
    // Halo piece i (of HALO_DMA 1-KiB pieces) of tile t into buf: lane-linear LDS slots
    // s = i*64 + lane hold (pixel p = s>>3, chunk pc = s&7); the XOR swizzle is applied to the
    // SOURCE address; slots past the halo read out of range (-> 0) into the slack.
    auto halo_piece = [&](int t, unsigned base, int i) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const int s = i * 64 + lane;
        const int p = s >> 3, pc = s & 7;
        const int hr = p / HALO, hc = p - hr * HALO;
        const int c = pc ^ (hc & 7);
        const int gh = h0 + hr - 1, gw = w0 + hc - 1;
        const bool in = s < HP * 8 && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
        const int voff = in ? (((b * H + gh) * W + gw) * 64 + c * 8) * 2 : 0x7ffffff0;
        dma16(xr4, __builtin_amdgcn_readfirstlane(base + i * 1024), voff);
    };

    FEN_STAMP(0);
    const EpiConst<MT> ec = epi_consts<MT>(d, co0 + wc * MT * 16 + q * 4);
    int t = slot;
    if (t < ntiles)
        for (int i = wave; i < HALO_DMA; i += NW) halo_piece(t, lds_addr(hbuf), i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    FEN_STAMP(1);
    for (int k = 0; t < ntiles; ++k, t += nslot) {
        char* cur = hbuf + (k & 1) * HALO_SLOT;   // halo of tile t, then its output stage
        const int tn = t + nslot;
        const unsigned nbase = lds_addr(hbuf + ((k + 1) & 1) * HALO_SLOT);
        // the next tile's halo: all pieces up front, or (debug & 4) one piece per wave per tap
        const bool ilv = d.debug & 4;
        if (!ilv && tn < ntiles)
            for (int i = wave; i < HALO_DMA; i += NW) halo_piece(tn, nbase, i);
        auto next_halo = [&](int tap) {
            const int i = wave + tap * NW;
            if (ilv && tn < ntiles && i < HALO_DMA) halo_piece(tn, nbase, i);
        };
        f32x4 acc[MT][NT];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!(d.debug & 2)) {
            if (d.debug & 32) conv_tile_resident<T, COT, MT, NT>(acc, wts, cur, wr, wc, q, c16, next_halo);
            else conv_tile_rows<T, COT, MT, NT>(acc, wts, cur, wr, wc, q, c16);
        } else {
            for (int tap = 0; tap < 9; ++tap) next_halo(tap);
        }
        FEN_STAMP(2 + 3 * k);
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        int nst = 0;
        if (d.debug & 1) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n) asm volatile("" ::"v"(acc[m][n]));
        } else {
            nst = conv_epilogue<T, COT, WR, WC, EPIC, true>(d, acc, b, t, h0, w0, co0,
                                                               (d.debug & 64) ? nullptr : cur, red, ec);
        }
        FEN_STAMP(3 + 3 * k);
        wait_vm_upto(nst);                                   // next halo landed (stores may drain)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                        // ... for everyone; cur is free
        FEN_STAMP(4 + 3 * k);
    }
}

// ------------------------------------------------------------------------------------
// k_conv3x3_g: persistent, two wave-groups in ping-pong (16-bit, Cin == 64, Cout % 64 == 0).
// 512 threads = group A (waves 0-3) + group B (waves 4-7); each wave owns 4 output rows x
// 16 columns x all 64 output channels of a tile (16 accumulators, halo-row-reuse MFMA
// order).  The block's tiles alternate between the groups, and the groups alternate
// roles every phase: while one group runs the MFMAs of its tile (reading the shared,
// LDS-resident filter and its own halo slot), the other group retires its previous tile
// (epilogue + direct stores) and streams its next halo by LDS-DMA into its own slot.  One
// s_barrier per phase; nothing else synchronises.  The per-channel partial sums of a tile
// (SE pool / PReLU dalpha) are parked in LDS in the epilogue phase and folded into
// part[tile][co] by the same group at the start of its next phase.
//   LDS: filter 72 KB | halo slot A | halo slot B | red[2][4][64] | bias[64] alpha[64]
// ------------------------------------------------------------------------------------
constexpr int G_WBYTES = 9 * 64 * 128;
constexpr int G_LDS = G_WBYTES + 2 * HALO_SLOT + 2 * 4 * 64 * 4 + 2 * 64 * 4;

template <typename T, int EPIC>
__global__ __launch_bounds__(512, 1) void k_conv3x3_g(const fen_conv_desc d) {
    constexpr int MT = 4, NT = 4;
    constexpr int NRES = (EPIC >> 8) & 3;
    constexpr int EPI = EPIC & ~(0x300 | EPIC_MPOOL);
    constexpr bool MPOOL = EPIC & EPIC_MPOOL;
    constexpr bool PRELU = EPI & FEN_EPI_PRELU, PBWD = EPI & FEN_EPI_PRELU_BWD, POOL = EPI & FEN_EPI_POOL;
    constexpr bool RBWD = EPI & FEN_EPI_RELU_BWD;
    constexpr bool SHUF = EPI & FEN_EPI_SHUFFLE, DOT = EPI & FEN_EPI_DOT;
    constexpr bool PART = POOL || PBWD || DOT;                // per-tile channel partials
    constexpr bool PIN = PBWD || DOT || RBWD;                 // reads pre_in
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wts = smem;
    float* red = (float*)(smem + G_WBYTES + 2 * HALO_SLOT);   // [grp][wr][64]
    float* cst = red + 2 * 4 * 64;                            // bias[64], alpha[64]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave >> 2, wr = wave & 3;
    const int q = lane >> 4, c16 = lane & 15;
    const int H = d.H, W = d.W, Cout = d.Cout;
    const int ncot = Cout >> 6;
    const int bid = xcd_block();                             // a tile's co blocks + neighbours: one XCD
    const int cot = bid % ncot, co0 = cot * 64;
    const int nslot = gridDim.x / ncot, slot = bid / ncot;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int ntiles = d.B * tpi;
    const int nmine = (ntiles - slot + nslot - 1) / nslot;    // tiles of this block (>= 1)
    const int nj0 = (nmine + 1) >> 1, nj1 = nmine >> 1;      // per group
    const int myn = grp ? nj1 : nj0;
    char* hslot = smem + G_WBYTES + grp * HALO_SLOT;
    const i32x4 xr4 = make_rsrc(d.x, (unsigned)((size_t)d.B * H * W * 128));

    FEN_STAMP(0);
    auto tile_of = [&](int g, int j) { return slot + (2 * j + g) * nslot; };
    // this group's share of the 41 halo pieces of tile t into its slot
    auto issue_halo = [&](int t) {
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const unsigned base = lds_addr(hslot);
        for (int i = wr; i < HALO_DMA; i += 4) {
            const int s = i * 64 + lane;
            const int p = s >> 3, pc = s & 7;
            const int hr = p / HALO, hc = p - hr * HALO;
            const int c = pc ^ (hc & 7);
            const int gh = h0 + hr - 1, gw = w0 + hc - 1;
            const bool in = s < HP * 8 && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
            const int voff = in ? (((b * H + gh) * W + gw) * 64 + c * 8) * 2 : 0x7ffffff0;
            dma16(xr4, __builtin_amdgcn_readfirstlane(base + i * 1024), voff);
        }
    };

    // ---- start-up: filter slab of co-tile cot, bias/alpha, group A's first halo
    {
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)d.w, (short)0, (int)((size_t)9 * Cout * 128), 0x00020000);
        for (int i = wave; i < G_WBYTES / 1024; i += 8) {
            const int s = i * 64 + lane;
            const int r = s >> 3, pc = s & 7;
            const int c = pc ^ ((r >> 1) & 7);
            const int tap = r >> 6, col = r & 63;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void*)(wts + i * 1024), 16,
                                                     ((tap * Cout + co0 + col) * 64 + c * 8) * 2, 0, 0, 0);
        }
        // the halo DMA goes out before the constant loads: their LDS writes wait for vmcnt,
        // which counts in issue order -- placed first, wave 0's halo share waited for the slab
        if (grp == 0) issue_halo(tile_of(0, 0));
        if (tid < 64) {
            const int cp = co0 + tid, Cq = Cout >> 2;
            const int co = SHUF ? 4 * (cp % Cq) + cp / Cq : cp;
            cst[tid] = (EPI & FEN_EPI_BIAS) ? d.bias[co] : 0.f;
            cst[64 + tid] = (PRELU || PBWD) ? d.alpha[SHUF ? cp % Cq : cp] : 0.f;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    FEN_STAMP(1);
    // pre_elide: all 64 slopes of this block's channels > 0 -> y_pre is not written (the
    // backward recovers it from y); block-uniform, so the store counts stay wave-uniform
    bool wpre = PRELU && d.y_pre;
    if (wpre && d.pre_elide) {
        bool allpos = true;
        for (int i = 0; i < 64; ++i) allpos = allpos && cst[64 + i] > 0.f;
        wpre = !allpos;
    }

    const int pend = max(2 * nj0 - 1, 2 * nj1);              // last phase (an epilogue)
    f32x4 acc[MT][NT];
    int pending_part = -1;                                   // tile whose partials sit in red[grp]
    for (int ph = 0; ph <= pend; ++ph) {
        int nst = 0;
        if ((ph & 1) == grp) {
            // ---------------- compute phase: tile j = (ph - grp) / 2 ----------------
            if (PART && pending_part >= 0 && wr == 0) {
                const float* rg = red + grp * 256;
                d.part[(size_t)pending_part * Cout + co0 + lane] =
                    (rg[lane] + rg[64 + lane]) + (rg[128 + lane] + rg[192 + lane]);
            }
            pending_part = -1;
            const int j = (ph - grp) >> 1;
            if (j < myn) {
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
                conv_tile_rows2<T, 64, MT, NT>(acc, wts, hslot, wr, 0, q, c16);
            }
        } else {
            // ---------------- service phase: retire tile jp, stream tile jp + 1 ----------------
            // the next halo is issued first; the residual / pre-activation loads follow and
            // one vmcnt(0) retires both (completion is in order), then the epilogue runs and
            // its stores drain across the barrier
            const int jp = (ph - grp - 1) >> 1;                  // -1 for group B at phase 0
            const bool ret = ph > grp && jp >= 0 && jp < myn;
            if (jp + 1 < myn) issue_halo(tile_of(grp, jp + 1));
            uint2 rv[NRES > 0 ? NRES : 1][MT][NT];
            uint2 pv[PIN ? MT : 1][PIN ? NT : 1];
            int b = 0, h0 = 0, w0 = 0, t = 0;
            bool full = true;
            bool rec_m[MT];                                      // PBWD: pre-activation from post_in
#pragma unroll
            for (int m = 0; m < MT; ++m) rec_m[m] = PBWD && d.post_in && all_pos4(cst + 64 + m * 16 + 4 * q);
            if (ret) {
                t = tile_of(grp, jp);
                b = t / tpi;
                const int tile = t - b * tpi;
                h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
                full = h0 + 16 <= H && w0 + 16 <= W;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int h = h0 + wr * NT + n, w = w0 + c16;
                    const bool ok = full || (h < H && w < W);
                    const size_t oi = ((size_t)(b * H + (ok ? h : 0)) * W + (ok ? w : 0)) * Cout + co0 + 4 * q;
#pragma unroll
                    for (int m = 0; m < MT; ++m) {
#pragma unroll
                        for (int k = 0; k < NRES; ++k) rv[k][m][n] = *(const uint2*)((const char*)d.res[k] + (oi + m * 16) * 2);
                        if constexpr (PIN) {
                            const void* src = (PBWD && rec_m[m]) ? d.post_in : d.pre_in;
                            pv[m][n] = *(const uint2*)((const char*)src + (oi + m * 16) * 2);
                        }
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (ret) {
                float psum[MT][4];
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) psum[m][r] = 0.f;
                const int Cq = Cout >> 2;
                // pass 1 (in place): bias, residuals, PReLU backward, partial sums -- consumes
                // the loaded operands right away so their registers die before the stores
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const float4 bb = *(const float4*)(cst + m * 16 + 4 * q);
                    const float4 aa = *(const float4*)(cst + 64 + m * 16 + 4 * q);
                    const float bias4[4] = {bb.x, bb.y, bb.z, bb.w};
                    const float al4[4] = {aa.x, aa.y, aa.z, aa.w};
#pragma unroll
                    for (int n = 0; n < NT; ++n) {
                        const bool ok = full || (h0 + wr * NT + n < H && w0 + c16 < W);
                        const float okf = ok ? 1.f : 0.f;
                        float rf[NRES > 0 ? NRES : 1][4], pf[4];
#pragma unroll
                        for (int k = 0; k < NRES; ++k) {
                            rf[k][0] = lo16<T>(rv[k][m][n].x);
                            rf[k][1] = hi16<T>(rv[k][m][n].x);
                            rf[k][2] = lo16<T>(rv[k][m][n].y);
                            rf[k][3] = hi16<T>(rv[k][m][n].y);
                        }
                        if constexpr (PIN) {
                            pf[0] = lo16<T>(pv[m][n].x);
                            pf[1] = hi16<T>(pv[m][n].x);
                            pf[2] = lo16<T>(pv[m][n].y);
                            pf[3] = hi16<T>(pv[m][n].y);
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float v = acc[m][n][r] + bias4[r];
#pragma unroll
                            for (int k = 0; k < NRES; ++k) v += rf[k][r];
                            if constexpr (PBWD) {
                                const float pr = pf[r];
                                psum[m][r] += okf * prelu_dalpha_f(v, pr);
                                v = prelu_bwd_f(v, pr, al4[r]);
                            }
                            if constexpr (RBWD) v = pf[r] > 0.f ? v : 0.f;
                            if constexpr (POOL) psum[m][r] += okf * v;
                            if constexpr (DOT) psum[m][r] += okf * rnd16<T>(v) * pf[r];
                            acc[m][n][r] = v;
                        }
                    }
                }
                // pass 2: activation + stores
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const float4 aa = *(const float4*)(cst + 64 + m * 16 + 4 * q);
                    const float al4[4] = {aa.x, aa.y, aa.z, aa.w};
#pragma unroll
                    for (int n = 0; n < NT; ++n) {
                        const int h = h0 + wr * NT + n, w = w0 + c16;
                        if (!(full || (h < H && w < W))) continue;
                        float v[4], o[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            v[r] = acc[m][n][r];
                            o[r] = PRELU ? prelu_f(v[r], al4[r]) : v[r];
                        }
                        const int cob = co0 + m * 16 + 4 * q;
                        size_t off;
                        if constexpr (SHUF) {
                            const int tt = cob / Cq, c = cob % Cq;
                            off = ((size_t)(b * 2 * H + 2 * h + (tt >> 1)) * (2 * W) + 2 * w + (tt & 1)) * Cq + c;
                        } else {
                            off = ((size_t)(b * H + h) * W + w) * Cout + cob;
                        }
                        if (MPOOL && d.y_images > 0 && b >= d.y_images) continue;   // (block-uniform)
                        if (wpre) {
                            st4<T>((char*)d.y_pre + off * 2, v);
                            ++nst;
                        }
                        st4<T>((char*)d.y + off * 2, o);
                        ++nst;
                    }
                }
                if constexpr (MPOOL) {
                    pool2_store<T, MT>(d, b, h0 + wr * NT, w0, co0 + 4 * q, c16, full, [&](int m, int n, int r) {
                        return PRELU ? prelu_f(acc[m][n][r], cst[64 + m * 16 + 4 * q + r]) : acc[m][n][r];
                    });
                }
                if constexpr (PART) {
                    float* rg = red + grp * 256 + wr * 64;
#pragma unroll
                    for (int m = 0; m < MT; ++m)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            // PBWD from post_in: the slope partials were taken over the PReLU output
                            const float sv = group16_sum(psum[m][r]) *
                                             ((PBWD && rec_m[m]) ? __builtin_amdgcn_rcpf(cst[64 + m * 16 + 4 * q + r]) : 1.f);
                            if (c16 == 0) rg[m * 16 + 4 * q + r] = sv;
                        }
                    pending_part = t;
                }
                if (!full) nst = 0;
            }
        }
        FEN_STAMP(2 + 2 * ph);
        wait_vm_upto(nst);                 // this wave's halo pieces landed (stores may drain)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        FEN_STAMP(3 + 2 * ph);
    }
    if (PART && pending_part >= 0 && wr == 0) {
        const float* rg = red + grp * 256;
        d.part[(size_t)pending_part * Cout + co0 + lane] = (rg[lane] + rg[64 + lane]) + (rg[128 + lane] + rg[192 + lane]);
    }
}

// ------------------------------------------------------------------------------------
// k_conv3x3_s: streamed per-tap weights, register-staged halo (f32 / bf16 / fp16, any Cin panel)
// ------------------------------------------------------------------------------------
// halo chunks of the next Cin panel loaded during the current panel's taps (the rest after it)
#ifndef CONV_S_PFN
#define CONV_S_PFN 11
#endif
template <typename T, int COT, int EPIC = -1>
__global__ __launch_bounds__(256, 2) void k_conv3x3_s(const fen_conv_desc d) {
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
    const int tb = xcd_block();                // neighbouring tiles on one XCD (halo rows in its L2)
    const int b = tb / tpi, tile = tb - b * tpi;
    const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
    const int co0 = blockIdx.y * COT;
    const int coutp = (Cout + 15) & ~15;
    const char* xb = (const char*)d.x;
    const char* wb = (const char*)d.w;
    const size_t xrow = (size_t)Cin * sizeof(T);

    f32x4 acc[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    // a last partial panel (Cin % CK: FaceEnhanceNetLite's 32 channels in 16-bit) reads zeros
    // past Cin, in the halo and in the filter
    const int npan = (Cin + CK - 1) / CK;
    // space-to-depth stride-2 convs (fen_conv_desc.s2d_in / s2d_out): only the taps the
    // scattered filter fills, (1 + a)(1 + b) of 9 for phase (a, b) -- forward taps kh', kw' in
    // {1} u ({0} if the phase bit is set); the mode-2 (flipped) data gradient's in {1} u {2}
    auto live_taps = [&](int ph, bool flipped) -> unsigned {
        const unsigned r = (ph >> 1) ? (flipped ? 6u : 3u) : 2u;     // bit set of kh' (or kh'')
        const unsigned c = (ph & 1) ? (flipped ? 6u : 3u) : 2u;
        unsigned m = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t)
            if ((r >> (t / 3)) & (c >> (t % 3)) & 1u) m |= 1u << t;
        return m;
    };
    const unsigned mask_out = d.s2d_out > 0 ? live_taps(co0 / d.s2d_out, true) : 0x1ffu;
    // ---- the input halo of a panel (zero padding outside the image), through registers ----
    constexpr int HPT = (HP * 8 + 255) / 256;   // 11 chunks per thread
    uint4 hv[HPT];
    unsigned hok = 0;                           // bit j: chunk j in range (else stored as zeros)
    auto halo_load = [&](int pn, int j) {
        int t = tid;
        asm volatile("" : "+v"(t));             // addresses per call: not hoisted across the panels
        const int i = t + j * 256;
        const int p = i >> 3, ch = i & 7;
        const int hr = p / HALO, hc = p - hr * HALO;
        const int gh = h0 + hr - 1, gw = w0 + hc - 1;
        const bool ok = i < HP * 8 && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W &&
                        pn * 128 + ch * 16 < (int)xrow;
        // branch-free: an out-of-range chunk loads the image's first one and is zeroed after, so
        // the vmcnt bookkeeping sees the same loads on every path (a branch makes hipcc wait for
        // all of them at the next use of any)
        // the zeroing waits for the store (a select right behind the load would wait for it)
        const size_t off = ok ? ((size_t)(b * H + gh) * W + gw) * xrow + pn * 128 + ch * 16 : 0;
        hv[j] = *(const uint4*)(xb + off);
        hok = ok ? hok | (1u << j) : hok & ~(1u << j);
    };
    auto halo_store = [&]() {
#pragma unroll
        for (int j = 0; j < HPT; ++j) {
            const int i = tid + j * 256;
            const uint4 v = ((hok >> j) & 1u) ? hv[j] : make_uint4(0, 0, 0, 0);
            if (i < HP * 8) *(uint4*)(halo + hswz(i >> 3, i & 7)) = v;
        }
    };
#pragma unroll
    for (int j = 0; j < HPT; ++j) halo_load(0, j);
    // one Cin panel; NEXT: the next panel's halo loads are issued during this one (their
    // registers are free in the last panel, which loads the epilogue constants instead)
    auto run_panel = [&](int pn, auto NEXT) {
        constexpr bool next = decltype(NEXT)::value;
        const unsigned mask = d.s2d_in > 0 ? live_taps(pn * CK / d.s2d_in, false) : mask_out;
        halo_store();                           // panel pn (the loads were issued one panel ahead)
        uint4 wr[WPT];
        // every thread loads WPT chunks (chunk index wrapped, duplicates are harmless): no
        // per-load branch, so hipcc keeps the prefetch in flight across the tap's MFMAs
        auto load_w = [&](int tap) {
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const int i = (tid + j * 256) % WCH;
                const int r = i >> 3, ch = i & 7;
                wr[j] = pn * 128 + ch * 16 < (int)xrow
                            ? *(const uint4*)(wb + (size_t)(tap * coutp + co0 + r) * xrow + pn * 128 + ch * 16)
                            : make_uint4(0, 0, 0, 0);
            }
        };
        auto store_w = [&](char* dst) {
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const int i = (tid + j * 256) % WCH;
                *(uint4*)(dst + swz(i >> 3, i & 7)) = wr[j];
            }
        };
        // live taps in order (mask is block-uniform: scalar bit walk)
        unsigned rem = mask;
        int tap = __builtin_ctz(rem);
        rem &= rem - 1;
        load_w(tap);
        store_w(wbuf);
        __syncthreads();
        for (int it = 0;; ++it) {
            const bool more = rem != 0;
            const int ntap = more ? __builtin_ctz(rem) : 0;
            if (more) load_w(ntap);            // issue early, write after the MFMAs
            conv_tap<T, MT, 4>(acc, wbuf + (it & 1) * COT * 128, halo, tap, wave, 0, q, c16);
            if (more) store_w(wbuf + ((it + 1) & 1) * COT * 128);
            __syncthreads();
            if (!more) break;
            rem &= rem - 1;
            tap = ntap;
        }
        if (next) {
#pragma unroll
            for (int j = 0; j < HPT; ++j) halo_load(pn + 1, j);
        }
    };
#ifndef CONV_S_NOPF
    // Every tap live (no space-to-depth): the (panel, tap) steps as one pipeline.  Weights two
    // steps ahead (two register sets, step s + 2 issued during step s) into a
    // 3-slot LDS ring (step s in slot s % 3, 9 % 3 == 0: the slot is the tap's), so an L2 round
    // trip has two steps of MFMAs to land in and no panel starts on an exposed weight load; the
    // next panel's halo chunks ride under this panel's taps, one or two per tap, after that
    // tap's weight loads (a wait on the older weights leaves them in flight).
    const bool fast = d.s2d_in <= 0 && mask_out == 0x1ffu;
#else
    const bool fast = false;
#endif
    uint4 w2[2][WPT];   // step s + 1 in w2[(it + 1) & 1], step s + 2 loaded into w2[it & 1]
    auto ldw = [&](int pn, int tap, uint4 (&w)[WPT]) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int i = (tid + j * 256) % WCH;
            const int r = i >> 3, ch = i & 7;
            // branch-free as halo_load; a chunk past Cin (a last partial panel) re-reads chunk 0
            // of the row and is zeroed by stw
            const bool ok = pn * 128 + ch * 16 < (int)xrow;
            w[j] = *(const uint4*)(wb + (size_t)(tap * coutp + co0 + r) * xrow + (ok ? pn * 128 + ch * 16 : 0));
        }
    };
    auto stw = [&](const uint4 (&w)[WPT], char* dst, int pn) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int i = (tid + j * 256) % WCH;
            const bool ok = pn * 128 + (i & 7) * 16 < (int)xrow;
            *(uint4*)(dst + swz(i >> 3, i & 7)) = ok ? w[j] : make_uint4(0, 0, 0, 0);
        }
    };
    auto fast_panel = [&](int pn, auto NEXT) {
        constexpr bool next = decltype(NEXT)::value;
#pragma unroll
        for (int it = 0; it < 9; ++it) {
            if (it + 2 < 9) ldw(pn, it + 2, w2[it & 1]);
            else if (next) ldw(pn + 1, it - 7, w2[it & 1]);
            if (next) {
#pragma unroll
                for (int j = 0; j < CONV_S_PFN; ++j)
                    if (j * 9 / CONV_S_PFN == it) halo_load(pn + 1, j);
            }
            conv_tap<T, MT, 4>(acc, wbuf + (it % 3) * COT * 128, halo, it, wave, 0, q, c16);
            if (it < 8 || next) stw(w2[(it + 1) & 1], wbuf + ((it + 1) % 3) * COT * 128, it < 8 ? pn : pn + 1);
            __syncthreads();
        }
        if (next) {
#pragma unroll
            for (int j = CONV_S_PFN; j < HPT; ++j) halo_load(pn + 1, j);
            halo_store();
            // 9 steps per panel (odd): the next panel's tap 1 came into w2[0], its entry wants w2[1]
#pragma unroll
            for (int j = 0; j < WPT; ++j) w2[1][j] = w2[0][j];
            __syncthreads();
        }
    };
    if (fast) {
        ldw(0, 0, w2[0]);
        ldw(0, 1, w2[1]);
        halo_store();
        stw(w2[0], wbuf, 0);
        __syncthreads();
        for (int pn = 0; pn + 1 < npan; ++pn) fast_panel(pn, std::true_type{});
    } else {
        for (int pn = 0; pn + 1 < npan; ++pn) run_panel(pn, std::true_type{});
    }
    const EpiConst<MT> ec = epi_consts<MT>(d, co0 + q * 4);   // latency hidden by the last panel
    if (fast) fast_panel(npan - 1, std::false_type{});
    else run_panel(npan - 1, std::false_type{});
    float* red = (float*)wbuf;     // LDS is free after the loop
    char* stage = (sizeof(T) == 2 && COT == 64) ? halo : nullptr;
    conv_epilogue<T, COT, 4, 1, EPIC>(d, acc, b, tb, h0, w0, co0, stage, red, ec);
}

// ------------------------------------------------------------------------------------
// k_conv3x3_v: persistent, LDS-DMA-fed (16-bit, Cin % 64 == 0, Cin >= 128, Cout % 128 == 0):
// the wide convs of VGG19's perceptual extractor (perceptual.py:13-169: conv2_2 .. conv3_4 and
// their data gradients) and of the discriminator (discriminator.py:58-90), where the filter slab
// (9 x Cin x Cout) is far larger than the LDS, so it streams.
// 512 threads = 8 waves; a block owns 128 output channels (co-tile fixed per block, tiles
// strided over the blocks, XCD-aware); wave (wr, wc) = 4 output rows x 16 columns x 64 channels
// of the 16 x 16 tile (16 accumulators, the streamed kernel's wave shape).  The K loop of a tile
// is npan x 9 steps (64-channel Cin panel, tap), and the steps of consecutive tiles run as ONE
// pipeline.  Operands arrive by LDS-DMA only (nothing through VGPRs or ds_write): step s's 16-KB
// weight slab (128 co x 64 ci) into slot s % 4 of a ring, three steps ahead, issued by waves 4-7;
// each panel's 18 x 18 halo into one of two slots, a whole panel ahead, issued by waves 0-3.
// vmcnt counts a wave's own loads in issue order, so the split keeps a weight wave's wait for
// the next step's slab from also waiting for a halo that is not due for eight more steps.  One
// s_barrier per step certifies the NEXT step's operands (each wave first waits for its own
// pieces of them), so a step reads the next step's first k-half fragments under its own
// second-half MFMAs and its MFMAs start right behind the barrier.  Taps are unrolled: every LDS
// address is a per-lane constant plus a scalar slot base.
// LDS: ring 4 x 16 KB | halo 2 x 44 KB | epilogue partials 2 KB = 154 KB.
// ------------------------------------------------------------------------------------
constexpr int V_COT = 128;
constexpr int V_WSLOT = V_COT * 128;       // one (tap, panel) weight slab
constexpr int V_RING = 4;
constexpr int V_HPIECES = 44;              // 41 halo pieces rounded up to 11 per halo wave
constexpr int V_HSLOT = V_HPIECES * 1024;
constexpr int V_LDS = V_RING * V_WSLOT + 2 * V_HSLOT + 4 * V_COT * 4;
constexpr int V_BAD = 0x7f000000;          // a voffset past any buffer fen_conv3x3 routes here (loads 0)

template <typename T, int EPIC>
__global__ __launch_bounds__(512, 1) void k_conv3x3_v(const fen_conv_desc d) {
    constexpr int MT = 4, NT = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wring = smem;
    char* hbuf = smem + V_RING * V_WSLOT;
    float* red = (float*)(hbuf + 2 * V_HSLOT);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wv = wave_id();                                // the same, scalar: role branches are real branches
    const bool hwave = wv < 4;                               // halo DMA (0-3) / weight DMA (4-7)
    const int wl = wv & 3;
    const int wr = wave & 3, wc = wave >> 2;
    const int q = lane >> 4, c16 = lane & 15;
    const int H = d.H, W = d.W, Cin = d.Cin, Cout = d.Cout;
    const int ncot = Cout / V_COT;
    const int bid = xcd_block();
    const int cot = bid % ncot, co0 = cot * V_COT;
    const int nslot = gridDim.x / ncot, slot = bid / ncot;
    const int twn = (W + 15) >> 4, tpi = twn * ((H + 15) >> 4);
    const int ntiles = d.B * tpi;
    const int nmine = slot < ntiles ? (ntiles - slot + nslot - 1) / nslot : 0;
    const int npan = Cin >> 6;
    const int nsteps = nmine * npan * 9;
    if (nsteps == 0) return;                                 // block-uniform
    const i32x4 xr4 = make_rsrc(d.x, (unsigned)((size_t)d.B * H * W * Cin * 2));
    const i32x4 wr4 = make_rsrc(d.w, (unsigned)((size_t)9 * Cout * Cin * 2));

    // weight waves: per-lane source offsets of their 4 pieces (i = 4 wl + k) of a slab, less the
    // (tap, panel) term; the LDS slot is lane-linear, the XOR swizzle on the source chunk
    auto issue_w = [&](int slot_i, int tap, int pn) {
        const unsigned base = lds_addr(wring + slot_i * V_WSLOT) + 4 * wl * 1024;
        const int so = (tap * Cout + co0) * Cin * 2 + pn * 128;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sl = (4 * wl + k) * 64 + lane;
            const int r = sl >> 3, pc = sl & 7;
#ifndef CVX_NOW
            dma16(wr4, base + k * 1024, so + (r * Cin + (pc ^ ((r >> 1) & 7)) * 8) * 2);
#endif
        }
    };
    // halo waves: their 11 pieces (i = wl + 4 k) of tile t's halo, Cin panel pn, into slot par
    // (zero padding: a voffset past the buffer outside the image / past the 18 x 18 pixels)
    auto issue_hk = [&](int par, int t, int pn, int k) {     // piece k (< 11) of this wave's share
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const unsigned base = lds_addr(hbuf + par * V_HSLOT) + wl * 1024;
        const int sl = (wl + 4 * k) * 64 + lane;
        const int p = sl >> 3, pc = sl & 7;
        const int hr = p / HALO, hc = p - hr * HALO;
        const int gh = h0 + hr - 1, gw = w0 + hc - 1;
        const bool in = p < HP && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
        const int voff = in ? (((b * H + gh) * W + gw) * Cin + (pc ^ (hc & 7)) * 8) * 2 + pn * 128 : V_BAD;
#ifndef CVX_NOH
        dma16(xr4, __builtin_amdgcn_readfirstlane(base + k * 4096), voff);
#endif
    };
    auto issue_h = [&](int par, int t, int pn) {
#pragma unroll 1
        for (int k = 0; k < 11; ++k) issue_hk(par, t, pn, k);
    };
    // per-lane LDS read offsets: A rows wc*64 + m*16 + c16 of a slab (the swizzle key (row >> 1) & 7
    // does not depend on m or wc: m steps are immediates), B at halo column c16 + kw, row wr*4 + kh + n
    const int aoff0 = swz(wc * 64 + c16, q), aoff1 = swz(wc * 64 + c16, 4 + q);
    auto load = [&](int wslot, int par, int kh, int kw, int kk, uint4 (&A)[MT], uint4 (&Bf)[NT]) {
        const char* pa = wring + wslot * V_WSLOT + (kk ? aoff1 : aoff0);
#pragma unroll
        for (int m = 0; m < MT; ++m) A[m] = *(const uint4*)(pa + m * 2048);
        const char* pb = hbuf + par * V_HSLOT + hcol(c16 + kw, kk * 4 + q) + (wr * NT + kh) * (HALO * 128);
#pragma unroll
        for (int n = 0; n < NT; ++n) Bf[n] = *(const uint4*)(pb + n * (HALO * 128));
    };
    f32x4 acc[MT][NT];
    auto mma = [&](const uint4 (&A)[MT], const uint4 (&Bf)[NT]) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) mma16<T>(acc[m][n], A[m], Bf[n]);
    };


    // prologue: tile 0's panel-0 halo; slabs of steps 0..2
    if (hwave) {
        issue_h(0, slot, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int s = 0; s < 3 && s < nsteps; ++s) issue_w(s, s, 0);
        if (nsteps > 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (nsteps > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    uint4 A0[MT], B0[NT], A1[MT], B1[NT];
    load(0, 0, 0, 0, 0, A0, B0);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    int s = 0, gp = 0;                                       // global step / panel counters
    for (int j = 0; j < nmine; ++j) {
        for (int pn = 0; pn < npan; ++pn, ++gp) {
            const int par = gp & 1;
            // the step 3 ahead: (tap + 3) % 9 of this panel or the next (of the next tile)
            const int pn3 = pn + 1 < npan ? pn + 1 : 0;
#pragma unroll 1
            for (int kh = 0; kh < 3; ++kh) {
#pragma unroll   // (kw unrolled: 302 vs 327 us on VGG conv3_2, A/B r6)
            for (int kw = 0; kw < 3; ++kw, ++s) {
                const int tap = kh * 3 + kw;
                if (s + 1 < nsteps) {
                    // certify step s + 1 (its slab; at tap 8 the next panel's halo)
                    if (!hwave) {
                        // (after a tile's epilogue this also waits for its stores: letting them stay
                        // in flight took a runtime count whose registers spilled -- slower, A/B r6)
                        if (s + 2 < nsteps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    } else if (kw == 2 && kh == 2) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifndef CVX_NOBAR   // (diagnostic variants: timing only, wrong results)
                    __builtin_amdgcn_s_barrier();            // and: every wave is done with step s - 1
#endif
                    if (hwave) {
                        // the next panel's halo, into the slot panel gp - 1 used (free since this
                        // panel's first barrier): the wave's 11 pieces in three bursts, at taps 0,
                        // 3 and 6 (4 + 4 + 3; all 11 at tap 0 held the halo waves for one long step
                        // while the barrier kept the other waves waiting), landed by tap 8's vmcnt(0)
#ifndef CVX_HALO_BURST
                        // (each piece issued between the MFMAs of the step's first half instead, the
                        // weight waves' too: conv3_2 343 vs 313-321 us, dgrad 180-183 vs 166-170, A/B r6)
                        if (kw == 0 && gp + 1 < nmine * npan) {
                            const int tn = pn + 1 < npan ? slot + j * nslot : slot + (j + 1) * nslot;
                            const int pnn = pn + 1 < npan ? pn + 1 : 0;
                            const int k1 = kh < 2 ? 4 * kh + 4 : 11;
#pragma unroll 1
                            for (int k = 4 * kh; k < k1; ++k) issue_hk(par ^ 1, tn, pnn, k);
                        }
#else   // A/B: round 6's first form, every piece at tap 0
                        if (kw == 0 && kh == 0 && gp + 1 < nmine * npan) {
                            if (pn + 1 < npan) issue_h(par ^ 1, slot + j * nslot, pn + 1);
                            else issue_h(par ^ 1, slot + (j + 1) * nslot, 0);
                        }
#endif
                    } else if (s + 3 < nsteps) {
                        issue_w((s + 3) & 3, (tap + 3) % 9, tap + 3 < 9 ? pn : pn3);   // into slot (s - 1) % 4
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                load(s & 3, par, kh, kw, 1, A1, B1);
                __builtin_amdgcn_sched_barrier(0);
                mma(A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                // the next step's first-half fragments (not across a tile end: the epilogue's
                // registers come first, the next tile's first fragments are read after it)
                if (kw < 2) load((s + 1) & 3, par, kh, kw + 1, 0, A0, B0);
                else if (kh < 2) load((s + 1) & 3, par, kh + 1, 0, 0, A0, B0);
                else if (pn + 1 < npan) load((s + 1) & 3, par ^ 1, 0, 0, 0, A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                mma(A1, B1);
                __builtin_amdgcn_sched_barrier(0);
            }
            }
        }
        // tile done: epilogue from registers (direct stores)
        const int t = slot + j * nslot;
        const int b = t / tpi, tile = t - b * tpi;
        const int h0 = (tile / twn) << 4, w0 = (tile % twn) << 4;
        const EpiConst<MT> ec = epi_consts<MT>(d, co0 + wc * 64 + q * 4);   // (per tile: 32 VGPRs less in the loop)
#ifndef CVX_NOEPI
        conv_epilogue<T, V_COT, 4, 2, EPIC, true>(d, acc, b, t, h0, w0, co0, nullptr, red, ec);
#else
        if (acc[0][0][0] == 12345.f) conv_epilogue<T, V_COT, 4, 2, EPIC, true>(d, acc, b, t, h0, w0, co0, nullptr, red, ec);
#endif
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (s < nsteps) load(s & 3, gp & 1, 0, 0, 0, A0, B0);   // the next tile's step 0 (certified)
    }
}

int g_num_cus = 0;

// kernel-variant selector for A/B runs (FEN_CONV_VARIANT): 0 default (ping-pong persistent
// kernel k_conv3x3_g for the network's epilogue modes), 1 streamed kernel everywhere,
// 2 single-group persistent kernel with the generic (runtime-mode) epilogue, 5 single-group
// persistent kernel k_conv3x3_p with per-mode epilogues
int conv_variant() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("FEN_CONV_VARIANT");
        v = e ? atoi(e) : 0;
    }
    return v;
}

template <typename T, int COT, int WR, int WC, int EPIC>
int launch_p(const fen_conv_desc* d, hipStream_t s) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int ntiles = d->B * tpi;
    const int ncot = ((d->Cout + 15) & ~15) / COT;
    if (g_num_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    int grid = g_num_cus;
    grid -= grid % ncot;
    const int maxg = ntiles * ncot;
    if (grid > maxg) grid = maxg;
    const size_t lds = 9 * COT * 128 + 2 * HALO_SLOT + WR * COT * 4 + 64;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_conv3x3_p<T, COT, WR, WC, EPIC>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr_set = true;
    }
    hipLaunchKernelGGL((k_conv3x3_p<T, COT, WR, WC, EPIC>), dim3(grid), dim3(64 * WR * WC), lds, s, *d);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

template <typename T, int EPIC>
int launch_g(const fen_conv_desc* d, hipStream_t s) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int ntiles = d->B * tpi;
    const int ncot = d->Cout / 64;
    if (g_num_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    int grid = g_num_cus;
    grid -= grid % ncot;
    const int maxg = ntiles * ncot;
    if (grid > maxg) grid = maxg;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_conv3x3_g<T, EPIC>, hipFuncAttributeMaxDynamicSharedMemorySize, G_LDS);
        attr_set = true;
    }
    hipLaunchKernelGGL((k_conv3x3_g<T, EPIC>), dim3(grid), dim3(512), G_LDS, s, *d);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

template <typename T, int EPIC>
int launch_v(const fen_conv_desc* d, hipStream_t s) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int ntiles = d->B * tpi;
    const int ncot = d->Cout / V_COT;
    if (g_num_cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    int grid = g_num_cus;
    grid -= grid % ncot;
    if (grid < ncot) grid = ncot;
    const int maxg = ntiles * ncot;
    if (grid > maxg) grid = maxg;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_conv3x3_v<T, EPIC>, hipFuncAttributeMaxDynamicSharedMemorySize, V_LDS);
        attr_set = true;
    }
    hipLaunchKernelGGL((k_conv3x3_v<T, EPIC>), dim3(grid), dim3(512), V_LDS, s, *d);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// the DMA-fed wide conv: 16-bit, Cin a multiple of 64 above 64, Cout of 128, stride 1, no
// (un)shuffle / conv_last, 32-bit buffer offsets (FEN_CONV_V=0: the streamed kernel instead)
bool conv_v_ok(const fen_conv_desc* d) {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("FEN_CONV_V");
        on = e ? atoi(e) : 1;
    }
    // (and enough 16 x 16 x 128 work items to fill the CUs: a long K loop on a quarter of the
    // chip lost to the streamed kernel's 2-blocks-per-CU grid -- the discriminator's 16 x 16 layers)
    const int items = d->B * ((d->H + 15) >> 4) * ((d->W + 15) >> 4) * (d->Cout / V_COT);
    int ncu = g_num_cus;
    if (ncu == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (ncu <= 0) ncu = 256;
        g_num_cus = ncu;
    }
    return on && conv_variant() != 1 && items >= ncu && d->Cin % 64 == 0 && d->Cin >= 128 && d->Cout % V_COT == 0 &&
           d->s2d_in == 0 && d->s2d_out == 0 && !(d->epi & (FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE | FEN_EPI_LAST)) &&
           (size_t)d->B * d->H * d->W * d->Cin * 2 < (size_t)V_BAD && (size_t)9 * d->Cout * d->Cin * 2 < (size_t)V_BAD;
}

template <typename T, int COT, int EPIC = -1>
int launch_s(const fen_conv_desc* d, hipStream_t s) {
    const int tpi = ((d->W + 15) >> 4) * ((d->H + 15) >> 4);
    const int coutp = (d->Cout + 15) & ~15;
    dim3 grid(d->B * tpi, coutp / COT);
    const size_t lds = HALO_BYTES + 3 * COT * 128;   // > 64 KB at COT = 64: opt in once
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_conv3x3_s<T, COT, EPIC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr_set = true;
    }
    hipLaunchKernelGGL((k_conv3x3_s<T, COT, EPIC>), grid, dim3(256), lds, s, *d);
    FEN_CHECK_LAUNCH();
    return FEN_OK;
}

// Kernel selection for one compute dtype T (float, bf16 or f16)
template <typename T>
int conv_dispatch(const fen_conv_desc* d, hipStream_t s) {
    const int epi = d->epi;
    constexpr bool H16 = sizeof(T) == 2;
    // the persistent kernels address the input with 32-bit buffer offsets
    const bool small = (size_t)d->B * d->H * d->W * 128 < (size_t)0x7fff0000;
    const bool s2d = d->s2d_in > 0 || d->s2d_out > 0;
    const bool persist = H16 && d->Cin == 64 && small && !(epi & FEN_EPI_UNSHUFFLE) && conv_variant() != 1 && !s2d;
    if (epi & FEN_EPI_LAST) {
        if (d->Cout > 4 || !d->lr || d->scale <= 0 || d->H % d->scale || d->W % d->scale) return FEN_EINVAL;
        if (epi & ~(FEN_EPI_LAST | FEN_EPI_BIAS)) return FEN_EUNSUPPORTED;
        if (fen_detail::conv_last_fast_ok(d) && conv_variant() != 1) return fen_detail::launch_conv_last(d, s);
        return launch_s<T, 16>(d, s);
    }
    if (!d->y) return FEN_EINVAL;
    if (epi & FEN_EPI_SHUFFLE) {
        if (d->Cout % 64) return FEN_EUNSUPPORTED;
        if (epi & (FEN_EPI_PRELU_BWD | FEN_EPI_POOL | FEN_EPI_DOT) || d->res[0] || d->res[1] || d->res[2])
            return FEN_EUNSUPPORTED;
    }
    if ((epi & FEN_EPI_UNSHUFFLE) && ((d->H | d->W) & 1)) return FEN_EINVAL;
    if (d->y_pool) {
        // the fused 2x2 max pool: bias + ReLU/PReLU stores of the persistent kernels; any other
        // route stores every image of y and pools it in a k_maxpool2 pass
        if constexpr (H16) {
            constexpr int B_ = FEN_EPI_BIAS;
            const bool dense = !d->res[0] && !d->res[1] && !d->res[2];
            if (dense && epi == (B_ | FEN_EPI_PRELU) && d->Cout % 64 == 0 && conv_variant() == 0) {
                if (persist) return launch_g<T, B_ | FEN_EPI_PRELU | EPIC_MPOOL>(d, s);
                if (conv_v_ok(d)) return launch_v<T, B_ | FEN_EPI_PRELU | EPIC_MPOOL>(d, s);
            }
        }
        fen_conv_desc d2 = *d;
        d2.y_pool = nullptr;
        d2.y_images = 0;
        const int rc = conv_dispatch<T>(&d2, s);
        if (rc != FEN_OK) return rc;
        return fen_maxpool2(d->dtype, d->B, d->H, d->W, d->Cout, d->y, d->y_pool, s);
    }
    if (d->Cout % 64 == 0) {
        if constexpr (H16) {
            if (persist) {
                // the network's epilogue modes get their own instantiation (mode | #residuals << 8)
                const int nres = d->res[0] ? (d->res[1] ? (d->res[2] ? 3 : 2) : 1) : 0;
                bool dense = true;   // residual pointers packed at the front
                for (int k = nres; k < 3; ++k) dense = dense && !d->res[k];
                const int key = dense && conv_variant() != 2 ? (epi | (nres << 8)) : -1;
                constexpr int B_ = FEN_EPI_BIAS;
                if (conv_variant() == 3 && key == (B_ | FEN_EPI_PRELU)) return launch_p<T, 64, 4, 1, B_ | FEN_EPI_PRELU>(d, s);
                if (conv_variant() != 5 && conv_variant() != 3) {
                    // default: the ping-pong kernel, except where the one-group persistent kernel
                    // measures faster (pool epilogue 19.2 vs 20.4 us, PReLU-backward 21.8 vs
                    // 36.3 us at B=32 64x64: the latter's register-heavy epilogue does not fit
                    // the ping-pong kernel's half-size register budget)
                    switch (key) {
                        case B_ | FEN_EPI_PRELU: return launch_g<T, B_ | FEN_EPI_PRELU>(d, s);
                        case B_ | FEN_EPI_POOL: return launch_p<T, 64, 4, 2, B_ | FEN_EPI_POOL>(d, s);
                        case B_ | (1 << 8): return launch_g<T, B_ | (1 << 8)>(d, s);
                        case B_ | FEN_EPI_PRELU | FEN_EPI_SHUFFLE: return launch_g<T, B_ | FEN_EPI_PRELU | FEN_EPI_SHUFFLE>(d, s);
                        case FEN_EPI_PRELU_BWD: return launch_p<T, 64, 4, 2, FEN_EPI_PRELU_BWD>(d, s);
                        case FEN_EPI_RELU_BWD: return launch_g<T, FEN_EPI_RELU_BWD>(d, s);
                        case 0: return launch_g<T, 0>(d, s);
                        case 1 << 8: return launch_g<T, 1 << 8>(d, s);
                        case 2 << 8: return launch_g<T, 2 << 8>(d, s);
                        case 3 << 8: return launch_g<T, 3 << 8>(d, s);
                        case FEN_EPI_DOT: return launch_g<T, FEN_EPI_DOT>(d, s);
                        case FEN_EPI_DOT | (1 << 8): return launch_g<T, FEN_EPI_DOT | (1 << 8)>(d, s);
                        default: break;
                    }
                }
                switch (key) {
                    case B_ | FEN_EPI_PRELU: return launch_p<T, 64, 4, 2, B_ | FEN_EPI_PRELU>(d, s);
                    case B_ | FEN_EPI_POOL: return launch_p<T, 64, 4, 2, B_ | FEN_EPI_POOL>(d, s);
                    case B_ | (1 << 8): return launch_p<T, 64, 4, 2, B_ | (1 << 8)>(d, s);
                    case B_ | FEN_EPI_PRELU | FEN_EPI_SHUFFLE:
                        return launch_p<T, 64, 4, 2, B_ | FEN_EPI_PRELU | FEN_EPI_SHUFFLE>(d, s);
                    case FEN_EPI_PRELU_BWD: return launch_p<T, 64, 4, 2, FEN_EPI_PRELU_BWD>(d, s);
                    case 0: return launch_p<T, 64, 4, 2, 0>(d, s);
                    case 1 << 8: return launch_p<T, 64, 4, 2, 1 << 8>(d, s);
                    case 2 << 8: return launch_p<T, 64, 4, 2, 2 << 8>(d, s);
                    case 3 << 8: return launch_p<T, 64, 4, 2, 3 << 8>(d, s);
                    default: return launch_p<T, 64, 4, 2, -1>(d, s);
                }
            }
        }
        if constexpr (H16) {
            if (conv_v_ok(d)) {
                const int nres = d->res[0] ? (d->res[1] ? (d->res[2] ? 3 : 2) : 1) : 0;
                bool dense = true;
                for (int k = nres; k < 3; ++k) dense = dense && !d->res[k];
                constexpr int B_ = FEN_EPI_BIAS;
                switch (dense ? (epi | (nres << 8)) : -1) {
                    case B_ | FEN_EPI_PRELU: return launch_v<T, B_ | FEN_EPI_PRELU>(d, s);
                    case B_: return launch_v<T, B_>(d, s);
                    case FEN_EPI_PRELU_BWD: return launch_v<T, FEN_EPI_PRELU_BWD>(d, s);
                    case FEN_EPI_RELU_BWD: return launch_v<T, FEN_EPI_RELU_BWD>(d, s);
                    case 0: return launch_v<T, 0>(d, s);
                    default: break;   // (the runtime-mode epilogue spills at this wave shape: streamed kernel)
                }
            }
        }
        if constexpr (H16) {
            // the upsampler dgrads (Cin = 4C): their epilogue modes as compile-time constants (no
            // residual loads or other modes' code in the epilogue's register budget)
#ifndef CONV_S_GENERIC   // A/B only: every streamed conv on the runtime-mode epilogue
            if (!d->res[0] && !d->res[1] && !d->res[2] && !s2d) {
                if (epi == (FEN_EPI_PRELU_BWD | FEN_EPI_UNSHUFFLE))
                    return launch_s<T, 64, FEN_EPI_PRELU_BWD | FEN_EPI_UNSHUFFLE>(d, s);
                if (epi == 0) return launch_s<T, 64, 0>(d, s);
            }
#endif
        }
        return launch_s<T, 64>(d, s);
    }
    // (Cout 16 from Cin 64 -- VGG conv1_1's data gradient -- on the one-group persistent kernel
    // with a 16-row resident filter measured 149 us vs the streamed kernel's 123 at B = 32, 256^2:
    // its per-tile residual loads and halo wait are exposed; r6)
    if (d->Cout % 16 == 0) return launch_s<T, 16>(d, s);
    return FEN_EUNSUPPORTED;
}

}  // namespace

extern "C" int fen_conv3x3(const fen_conv_desc* d, void* stream) {
    if (!d || !d->x || !d->w || d->B <= 0 || d->H <= 0 || d->W <= 0 || d->Cin <= 0 || d->Cout <= 0)
        return FEN_EINVAL;
    if (d->dtype != FEN_F32 && d->dtype != FEN_BF16 && d->dtype != FEN_F16) return FEN_EINVAL;
    // 16-B channel chunks: Cin % 8 (16-bit) / % 4 (f32); Cin == 64 takes the persistent kernels
    if ((d->Cin * (d->dtype == FEN_F32 ? 4 : 2)) % 16) return FEN_EUNSUPPORTED;
    const int epi = d->epi;
    if ((epi & FEN_EPI_BIAS) && !d->bias) return FEN_EINVAL;
    if ((epi & (FEN_EPI_PRELU | FEN_EPI_PRELU_BWD)) && !d->alpha) return FEN_EINVAL;
    if ((epi & (FEN_EPI_PRELU_BWD | FEN_EPI_DOT | FEN_EPI_RELU_BWD)) && !d->pre_in) return FEN_EINVAL;
    if (epi & ~0x10ff) return FEN_EINVAL;
    if ((epi & FEN_EPI_RELU_BWD) &&
        (epi & (FEN_EPI_PRELU_BWD | FEN_EPI_DOT | FEN_EPI_LAST | FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE)))
        return FEN_EUNSUPPORTED;
    if ((epi & (FEN_EPI_POOL | FEN_EPI_PRELU_BWD | FEN_EPI_DOT)) && !d->part) return FEN_EINVAL;
    if (d->y_images < 0 || d->y_images > d->B || (d->y_images && !d->y_pool)) return FEN_EINVAL;
    if (d->y_pool && (!(epi & FEN_EPI_PRELU) || ((d->H | d->W) & 1) || d->s2d_in || d->s2d_out ||
                      (epi & (FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE | FEN_EPI_LAST | FEN_EPI_POOL | FEN_EPI_DOT))))
        return FEN_EUNSUPPORTED;
    // one partial-sum stream per launch
    {
        const int np = !!(epi & FEN_EPI_POOL) + !!(epi & FEN_EPI_PRELU_BWD) + !!(epi & FEN_EPI_DOT);
        if (np > 1) return FEN_EUNSUPPORTED;
    }
    if ((epi & FEN_EPI_DOT) && (epi & (FEN_EPI_UNSHUFFLE | FEN_EPI_LAST))) return FEN_EUNSUPPORTED;
    // space-to-depth stride-2 form: whole 64-channel panels / output tiles per phase
    if (d->s2d_in < 0 || d->s2d_out < 0 || (d->s2d_in && d->s2d_out)) return FEN_EINVAL;
    if (d->s2d_in && (d->s2d_in % 64 || d->Cin != 4 * d->s2d_in)) return FEN_EINVAL;
    if (d->s2d_out && (d->s2d_out % 64 || d->Cout != 4 * d->s2d_out)) return FEN_EINVAL;
    if ((d->s2d_in || d->s2d_out) && (epi & (FEN_EPI_LAST | FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE)))
        return FEN_EUNSUPPORTED;
    if ((epi & (FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE)) == (FEN_EPI_SHUFFLE | FEN_EPI_UNSHUFFLE))
        return FEN_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    switch (d->dtype) {
        case FEN_BF16: return conv_dispatch<bf16>(d, s);
        case FEN_F16: return conv_dispatch<f16>(d, s);
        default: return conv_dispatch<float>(d, s);
    }
}

// Shared pieces of the strip-resident ResidualGroup kernels (group_strip.hip: the forward,
// group_strip_bwd.hip: the backward): strip geometry, the LDS image swizzle, the accumulator-
// layout row helpers, the agent-scope polls and one 3-tap conv phase on MFMA.
#pragma once
#include "fen_common.h"

namespace gs {

constexpr int SR = 8;                         // rows per strip = waves per block
constexpr int SW = 64;                        // strip width = image width
constexpr int IC = SW + 2;                    // LDS image columns (zero column each side)
constexpr int IROW = IC * 128;                // 8448 B per LDS image row
constexpr int IMG_BYTES = (SR + 2) * IROW;    // 84480
constexpr int TAPB = 64 * 128;                // one filter tap [64 co][64 ci]
constexpr int ROWB = SW * 128;                // one strip row, 8 KB
constexpr int SPIN_MAX = 1 << 20;             // polls (~1.5 us each) before a wait gives up

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// 4 consecutive channels (acc element order) <-> one 8-B word pair
template <typename T>
__device__ __forceinline__ uint2 pk4(float a, float b, float c, float d) {
    return make_uint2(pack2<T>(a, b), pack2<T>(c, d));
}

// lanes q and q^1 (same pixel: rows 2k, 2k+1 of 16 lanes) trade one 4-channel half so each
// holds 8 consecutive channels: lo = the lane's channels of m-block 2mp, hi = of m-block
// 2mp + 1; the result is chunk chunk_of(mp, q) of the pixel.  v_permlane16_swap swaps the odd
// rows of its first operand with the even rows of its second: even rows keep lo and receive
// the odd partner's lo, odd rows keep hi and receive the even partner's hi (no LDS round trip)
__device__ __forceinline__ uint4 pair16(uint2 lo, uint2 hi) {
    const auto a = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
    return make_uint4(a[0], b[0], a[1], b[1]);
}
__device__ __forceinline__ int chunk_of(int mp, int q) { return 4 * mp + ((q & 1) ? 2 : 0) + (q >> 1); }

// sum over the 8 lanes l ^ 8k (the lanes of one l & 7): row_ror:8 (lane ^ 8 in a row of 16),
// then the row-pair and half swaps; a fixed tree, bit-identical in all 8 lanes
__device__ __forceinline__ float sum_lanes_x8(float v) {
    v += dpp_f<0x128>(v);
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// P += sum_e bcast_e(v) * w[e], bcast_e = lane e of the lane's row of 16 (DPP row_newbcast)
template <int E>
__device__ __forceinline__ void bcast8_fma_(float& P, float v, const float (&w)[8]) {
    P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + E, 0xf, 0xf, false)) * w[E];
    if constexpr (E < 7) bcast8_fma_<E + 1>(P, v, w);
}
__device__ __forceinline__ void bcast8_fma(float& P, float v, const float (&w)[8]) { bcast8_fma_<0>(P, v, w); }

// bounded poll of an agent-scope flag (sc1 loads): true once it holds `tag`
__device__ __forceinline__ bool poll_eq(const unsigned* p, unsigned tag) {
    for (int it = 0; it < SPIN_MAX; ++it) {
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

// End of a strip launch, thread 0 of every block after its `ok` went into ctl[2] (drained):
// the last block out advances the launch epoch, resets the ticket counters for the next launch
// and, when the caller passed a status word, moves the error word there (a vector store at
// system scope: the word may be host-mapped pinned memory the host reads without a sync) and
// clears it, so a later launch on the same workspace starts clean.
// ctl: [0] ticket [1] done [2] error [3] launch epoch.
__device__ __forceinline__ void strip_finish(int* ctl, int nblk, int* status, int status_bit) {
    if (__hip_atomic_fetch_add(ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1) {
        if (status) {
            const int e = __hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e) {   // bit 0: a timed-out wait (status_bit); bit 1: a chain table mismatch
                __hip_atomic_store(status, ((e & 1) ? status_bit : 0) | ((e & 2) ? FEN_STATUS_GS_TABLE : 0),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(ctl + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __hip_atomic_fetch_add(ctl + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ void vm_wait_n(int n) {
    switch (n) {
#define GS_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        GS_VMC(1) GS_VMC(2) GS_VMC(3) GS_VMC(4) GS_VMC(5) GS_VMC(6) GS_VMC(7) GS_VMC(8) GS_VMC(9) GS_VMC(10)
        GS_VMC(11) GS_VMC(12) GS_VMC(13) GS_VMC(14) GS_VMC(15) GS_VMC(16)
#undef GS_VMC
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// one phase of a conv: the 3 taps (kh, 0..2) on the wave's output row; B fragments from LDS
// image row (wave + kh) at column shift kw, A fragments from tap slot kh * 3 + kw.  Six
// (tap, k-half) steps, the next step's fragments read during the current step's 16 MFMAs.
template <typename T>
__device__ __forceinline__ void conv_phase(f32x4 (&acc)[4][4], const char* img, const char* filt, int kh, int wave,
                                           int q, int c16) {
    asm volatile("" : "+v"(q), "+v"(c16));   // opaque lane coordinates: addresses per phase
    const char* rowp = img + (wave + kh) * IROW;
    const char* slot0 = filt + kh * 3 * TAPB;
    uint4 A[2][4], Bf[2][4];
    // the swizzle keys depend on the lane only (16 m and 16 p leave them unchanged): one base
    // address per step, m and p as immediate offsets
    auto load = [&](int s, uint4 (&a)[4], uint4 (&b)[4]) {
        const int kw = s >> 1, chunk = (s & 1) * 4 + q;
        const char* ab = slot0 + kw * TAPB + c16 * 128 + ((chunk ^ ((c16 >> 1) & 7)) << 4);
        const char* bb = rowp + (c16 + kw) * 128 + ((chunk ^ ((c16 + kw) & 7)) << 4);
#ifdef GS_BURST
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = *(const uint4*)(ab + m * 2048);
#pragma unroll
        for (int p = 0; p < 4; ++p) b[p] = *(const uint4*)(bb + p * 2048);
#else
        // in the order the next step's MFMAs (m-major) consume them
        b[0] = *(const uint4*)bb;
        a[0] = *(const uint4*)ab;
#pragma unroll
        for (int p = 1; p < 4; ++p) b[p] = *(const uint4*)(bb + p * 2048);
#pragma unroll
        for (int m = 1; m < 4; ++m) a[m] = *(const uint4*)(ab + m * 2048);
#endif
    };
    load(0, A[0], Bf[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        if (s + 1 < 6) load(s + 1, A[(s + 1) & 1], Bf[(s + 1) & 1]);
#ifdef GS_BURST
        __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int p = 0; p < 4; ++p) mma16<T>(acc[m][p], A[s & 1][m], Bf[s & 1][p]);
#ifndef GS_BURST
        // the next step's 8 fragment reads one per MFMA, not as a burst ahead of the 16
        // MFMAs: a SIMD's two waves leave every barrier together, and two bursts at once
        // drained the matrix pipe
        if (s + 1 < 6) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        }
#endif
        __builtin_amdgcn_sched_barrier(0);
    }
}

}  // namespace gs

// Shared device helpers for the FaceEnhanceNet gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "fen.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// fp16: the reference's own mixed-precision dtype (torch.cuda.amp.autocast, trainer.py:18,227,460);
// same MFMA rate as bf16 on gfx950 with 3 more mantissa bits (11 vs 8)
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// Per-dtype constants.  Every LDS "panel" row is 128 B: 64 bf16 or 32 f32 channels.
template <typename T> struct Tr;
template <> struct Tr<float> { static constexpr int CK = 32; static constexpr int EPC = 4; };
template <> struct Tr<bf16>  { static constexpr int CK = 64; static constexpr int EPC = 8; };
template <> struct Tr<f16>   { static constexpr int CK = 64; static constexpr int EPC = 8; };

// Byte offset of 16-B chunk `chunk` (0..7) of row `p` in a 128-B-row LDS image.  The XOR
// key (p>>1)&7 puts 16 consecutive rows read at the same chunk on 16 distinct 16-B slots
// of the 256-B bank row, so ds_read_b128 fragment reads are conflict-free.
// XCD-aware block index of a 1-D grid: blocks b and b + 8 share an XCD (round-robin dispatch,
// observed -- MI355X_MICROARCH.md, workgroup dispatch), so b -> (b % 8) * (n / 8) + b / 8 gives
// consecutive logical indices -- neighbouring tiles, or the output-channel blocks of one tile --
// one XCD and its L2.  Identity when n is not a multiple of 8.  A permutation: it moves
// traffic, never results.
__device__ __forceinline__ int xcd_block() {
    const int b = (int)blockIdx.x, n = (int)gridDim.x;
    return (n & 7) ? b : (b & 7) * (n >> 3) + (b >> 3);
}
__device__ __forceinline__ int swz(int p, int chunk) {
    return (p << 7) + ((chunk ^ ((p >> 1) & 7)) << 4);
}

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
    bf16 h = (bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN-preserving
    return __builtin_bit_cast(unsigned short, h);
}

// 16-bit pairs in one 32-bit word (element 0 in the low half): the bf16 forms are shifts,
// the fp16 forms hardware conversions (v_cvt_f32_f16 / v_cvt_pk_f16_f32-style RNE)
template <typename T> __device__ __forceinline__ float lo16(unsigned w);
template <typename T> __device__ __forceinline__ float hi16(unsigned w);
template <> __device__ __forceinline__ float lo16<bf16>(unsigned w) { return __uint_as_float(w << 16); }
template <> __device__ __forceinline__ float hi16<bf16>(unsigned w) { return __uint_as_float(w & 0xffff0000u); }
// fp16 halves through a 2-vector: v_cvt_f32_f16 (the high half via SDWA word select, one
// instruction) and v_cvt_pk_f16_f32 (two floats, one instruction, round-to-nearest-even)
template <> __device__ __forceinline__ float lo16<f16>(unsigned w) { return (float)__builtin_bit_cast(f16x2, w).x; }
template <> __device__ __forceinline__ float hi16<f16>(unsigned w) { return (float)__builtin_bit_cast(f16x2, w).y; }
template <typename T> __device__ __forceinline__ unsigned short to16(float f);
template <> __device__ __forceinline__ unsigned short to16<bf16>(float f) { return f2bf(f); }
template <> __device__ __forceinline__ unsigned short to16<f16>(float f) { return __builtin_bit_cast(unsigned short, (f16)f); }
template <typename T> __device__ __forceinline__ unsigned pack2(float lo, float hi) {
    return (unsigned)to16<T>(lo) | ((unsigned)to16<T>(hi) << 16);
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <> __device__ __forceinline__ unsigned pack2<f16>(float lo, float hi) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){lo, hi}, f16x2));
}

template <typename T> __device__ __forceinline__ float tof(T v);
template <> __device__ __forceinline__ float tof<float>(float v) { return v; }
template <> __device__ __forceinline__ float tof<bf16>(bf16 v) { return (float)v; }
template <> __device__ __forceinline__ float tof<f16>(f16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T fromf(float v);
// v as stored in T (the value a later pass would read back)
template <typename T> __device__ __forceinline__ float rnd16(float v);
template <> __device__ __forceinline__ float fromf<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 fromf<bf16>(float v) { return (bf16)v; }
template <> __device__ __forceinline__ f16 fromf<f16>(float v) { return (f16)v; }
template <> __device__ __forceinline__ float rnd16<float>(float v) { return v; }
template <> __device__ __forceinline__ float rnd16<bf16>(float v) { return (float)(bf16)v; }
template <> __device__ __forceinline__ float rnd16<f16>(float v) { return (float)(f16)v; }

// 4 consecutive elements <-> float[4]
template <typename T> __device__ __forceinline__ void ld4(const void* p, float v[4]);
template <> __device__ __forceinline__ void ld4<float>(const void* p, float v[4]) {
    float4 x = *(const float4*)p;
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
template <> __device__ __forceinline__ void ld4<bf16>(const void* p, float v[4]) {
    uint2 x = *(const uint2*)p;
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
}
template <> __device__ __forceinline__ void ld4<f16>(const void* p, float v[4]) {
    uint2 x = *(const uint2*)p;
    v[0] = lo16<f16>(x.x); v[1] = hi16<f16>(x.x);
    v[2] = lo16<f16>(x.y); v[3] = hi16<f16>(x.y);
}
template <typename T> __device__ __forceinline__ void st4(void* p, const float v[4]);
template <> __device__ __forceinline__ void st4<float>(void* p, const float v[4]) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void st4<bf16>(void* p, const float v[4]) {
    uint2 x;
    x.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    x.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    *(uint2*)p = x;
}

template <> __device__ __forceinline__ void st4<f16>(void* p, const float v[4]) {
    *(uint2*)p = make_uint2(pack2<f16>(v[0], v[1]), pack2<f16>(v[2], v[3]));
}

// 16-B vector of EPC elements <-> float[EPC]
template <typename T> __device__ __forceinline__ void unpack16(const uint4& u, float* v);
template <> __device__ __forceinline__ void unpack16<float>(const uint4& u, float* v) {
    v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y);
    v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
}
template <> __device__ __forceinline__ void unpack16<bf16>(const uint4& u, float* v) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
template <> __device__ __forceinline__ void unpack16<f16>(const uint4& u, float* v) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = lo16<f16>(w[i]);
        v[2 * i + 1] = hi16<f16>(w[i]);
    }
}
template <typename T> __device__ __forceinline__ uint4 pack16(const float* v);
template <> __device__ __forceinline__ uint4 pack16<float>(const float* v) {
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                      __float_as_uint(v[3]));
}
template <> __device__ __forceinline__ uint4 pack16<bf16>(const float* v) {
    uint4 u;
    u.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    u.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    u.z = (unsigned)f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
    u.w = (unsigned)f2bf(v[6]) | ((unsigned)f2bf(v[7]) << 16);
    return u;
}

template <> __device__ __forceinline__ uint4 pack16<f16>(const float* v) {
    return make_uint4(pack2<f16>(v[0], v[1]), pack2<f16>(v[2], v[3]), pack2<f16>(v[4], v[5]), pack2<f16>(v[6], v[7]));
}

// acc += A * B for one 16-byte fragment pair: one 16x16x32 bf16 MFMA, or four
// 16x16x4 f32 MFMAs (exact f32; element s of the 16 B is the k-step s).
template <typename T> __device__ __forceinline__ void mma16(f32x4& acc, const uint4& a, const uint4& b);
template <> __device__ __forceinline__ void mma16<bf16>(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <> __device__ __forceinline__ void mma16<f16>(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
}
template <> __device__ __forceinline__ void mma16<float>(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}

// PReLU in arithmetic form (torch's own definition: max(0,v) + a*min(0,v)) and its backward
// factor; written without a data-dependent select so hipcc never turns them into exec-masked
// branches that sink an operand's pending LDS/global read into the branch (measured: a
// 48-element epilogue became ~1000 instructions and ~2 us).
__device__ __forceinline__ float prelu_f(float v, float a) { return fmaxf(v, 0.f) + a * fminf(v, 0.f); }
__device__ __forceinline__ float pos_step(float v) { return v > 0.f ? 1.f : 0.f; }
// dy * dPReLU(pre)/dpre = dy * (pre > 0 ? 1 : a): one compare, one select, one multiply
__device__ __forceinline__ float prelu_bwd_f(float dy, float pre, float a) { return dy * (pre > 0.f ? 1.f : a); }
// contribution to dL/da: dy * pre where pre <= 0 (the compare above reused, one select)
__device__ __forceinline__ float prelu_dalpha_f(float dy, float pre) { return dy * (pre > 0.f ? 0.f : pre); }
__device__ __forceinline__ bool all_pos4(const float* a) { return a[0] > 0.f && a[1] > 0.f && a[2] > 0.f && a[3] > 0.f; }

// The wave index, provably wave-uniform to the compiler (threadIdx.x >> 6 alone is divergent
// to hipcc: every per-wave role built on it compiles to exec-masked code that all waves issue)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// sum over the 16 lanes of a DPP row (lanes 16r..16r+15), the same value in every lane:
// quad xor 1, quad xor 2, half-row mirror, row mirror -- VALU-only (no LDS round trips)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float group16_sum(float v) {
    v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);    // row_half_mirror
    v += dpp_f<0x140>(v);    // row_mirror
    return v;
}

// Keys cubic convolution, A = -0.75 (torch upsample_bicubic2d coefficients)
__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
    const float A = -0.75f;
    float x1 = t + 1.0f;
    c[0] = ((A * x1 - 5.0f * A) * x1 + 8.0f * A) * x1 - 4.0f * A;
    c[1] = ((A + 2.0f) * t - (A + 3.0f)) * t * t + 1.0f;
    float x2 = 1.0f - t;
    c[2] = ((A + 2.0f) * x2 - (A + 3.0f)) * x2 * x2 + 1.0f;
    float x3 = 2.0f - t;
    c[3] = ((A * x3 - 5.0f * A) * x3 + 8.0f * A) * x3 - 4.0f * A;
}

// Bicubic sample of plane img[hin][win] at output (oy, ox) for resize scale 1/inv_scale,
// align_corners=False, border-clamped taps; rows interpolated along x first, then along y.
__device__ __forceinline__ float bicubic_sample(const float* img, int hin, int win, int oy, int ox,
                                                float inv_scale) {
    float sy = ((float)oy + 0.5f) * inv_scale - 0.5f;
    float sx = ((float)ox + 0.5f) * inv_scale - 0.5f;
    float fy = floorf(sy), fx = floorf(sx);
    float cy[4], cx[4];
    cubic_coeffs(sy - fy, cy);
    cubic_coeffs(sx - fx, cx);
    int iy = (int)fy, ix = (int)fx;
    int xs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xs[j] = min(max(ix - 1 + j, 0), win - 1);
    float out = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float* row = img + (size_t)min(max(iy - 1 + i, 0), hin - 1) * win;
        float r = row[xs[0]] * cx[0] + row[xs[1]] * cx[1] + row[xs[2]] * cx[2] + row[xs[3]] * cx[3];
        out += r * cy[i];
    }
    return out;
}

// ---- 18x18 halo images and LDS-DMA helpers (gfx950 buffer_load ... lds) ----
constexpr int HALO = 18;
constexpr int HP = HALO * HALO;                // 324 halo pixels
constexpr int HALO_BYTES = HP * 128;           // 41472
constexpr int HALO_DMA = (HP * 8 + 63) / 64;   // 41 wave-wide 1-KiB LDS-DMA pieces per halo
constexpr int HALO_SLOT = HALO_DMA * 1024;     // 41984: halo + slack for the last piece

typedef __attribute__((address_space(3))) void lds_void;
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Halo images (18 x 18 pixels, 128-B rows): 16-B chunk c of pixel p sits at chunk c ^ (col & 7),
// col = p % 18.  Fragment reads touch 16 consecutive columns of one halo row at the same
// logical chunk -> 16 distinct 16-B bank slots (conflict-free ds_read_b128), and because the
// key depends only on the column, every read of a lane is base(kw, kk) + row * 2304.
__device__ __forceinline__ int hswz(int p, int chunk) {
    return (p << 7) + ((chunk ^ ((p % HALO) & 7)) << 4);
}
__device__ __forceinline__ int hcol(int col, int chunk) {   // offset of (column col, chunk) in a row
    return (col << 7) + ((chunk ^ (col & 7)) << 4);
}

// Buffer resource (V#) words for a raw byte buffer: base, stride 0, num_records = bytes.
// Loads at voffset >= bytes return 0 -- used for the conv's zero padding.
__device__ __forceinline__ i32x4 make_rsrc(const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
    r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32) & 0xffff);
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);
    r.w = 0x00020000;
    return r;
}

// 16 B per lane global -> LDS (buffer_load_dwordx4 ... lds) written to lds_base + lane*16.
// Issued from inline asm on purpose: hipcc then does not see an LDS write in flight, so it
// does not drain vmcnt before every ds_read of the *other* halo buffer.  The caller waits
// (s_waitcnt vmcnt(0)) and barriers before reading the destination.
__device__ __forceinline__ void dma16(const i32x4& rsrc, unsigned lds_base, int voff) {
    unsigned keep;  // M0 is compiler-reserved: save and restore it inside the statement
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(lds_base), "v"(voff), "s"(rsrc)
        : "memory");
}
// the same with the non-temporal cache policy (operands read once: no L2 / MALL allocation)
__device__ __forceinline__ void dma16_nt(const i32x4& rsrc, unsigned lds_base, int voff) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen nt lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(lds_base), "v"(voff), "s"(rsrc)
        : "memory");
}
// 4 B per lane (buffer_load_dword ... lds) written to lds_base + lane*4: gathers with
// per-element addresses (border-clamped patches)
__device__ __forceinline__ void dma4(const i32x4& rsrc, unsigned lds_base, int voff) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "buffer_load_dword %2, %3, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(lds_base), "v"(voff), "s"(rsrc)
        : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const lds_void*)p;
}

// hipGetLastError() also returns the last status of any HIP call made on this thread, so
// hipErrorNotReady left by a host-side hipEventQuery/hipStreamQuery (torch's gloo hand-off polls
// events between steps) is not a launch failure and is only consumed here.  A real failure is
// kept for fen_last_hip_error().
namespace fen_detail {
extern thread_local int last_hip_error;
}
#define FEN_CHECK_LAUNCH()                                        \
    do {                                                          \
        hipError_t e_ = hipGetLastError();                        \
        if (e_ != hipSuccess && e_ != hipErrorNotReady) {         \
            fen_detail::last_hip_error = (int)e_;                 \
            return FEN_EHIP;                                      \
        }                                                         \
    } while (0)

// conv_last fast path (conv_last.hip): bf16, Cin 64, Cout <= 4, x4 skip, H and W multiples of 16
namespace fen_detail {
bool conv_last_fast_ok(const fen_conv_desc* d);
int launch_conv_last(const fen_conv_desc* d, hipStream_t s);
}  // namespace fen_detail

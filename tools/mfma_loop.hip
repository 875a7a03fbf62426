// Microbenchmark: the conv kernel's LDS -> MFMA tap loop in isolation (no DMA, no epilogue).
// One persistent workgroup per CU re-runs the 9-tap x 2-k-half loop REPS times over fixed LDS
// images with the conv's exact address patterns, then reports the MFMA utilisation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_loop.hip -o tools/mfma_loop && tools/mfma_loop
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int HALO = 18;
__device__ __forceinline__ int swz(int p, int c) { return (p << 7) + ((c ^ ((p >> 1) & 7)) << 4); }
__device__ __forceinline__ int hcol(int col, int c) { return (col << 7) + ((c ^ (col & 7)) << 4); }
__device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                  0, 0, 0);
}

// WR x WC waves; wave tile = (64/WC) co x (16/WR rows of 16 px)
template <int WR, int WC, bool REGA>
__global__ __launch_bounds__(64 * WR * WC, 1) void k_loop(float* out, int reps) {
    constexpr int COT = 64, MT = COT / 16 / WC, NT = 16 / WR;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wts = smem;                       // 9 * 64 * 128
    char* halo = smem + 9 * COT * 128;      // 18*18*128
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave % WR, wc = wave / WR, q = lane >> 4, c16 = lane & 15;
    for (int i = tid; i < (9 * COT * 128 + HALO * HALO * 128) / 4; i += blockDim.x)
        ((unsigned*)smem)[i] = 0x3c003c00u ^ (i * 2654435761u & 0x00ff00ffu);
    __syncthreads();
    f32x4 acc[MT][NT];
    for (int m = 0; m < MT; ++m)
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0, 0, 0, 0};
    const int arow = wc * MT * 16 + c16;
    uint4 Areg[REGA ? 9 : 1][2][MT];
    if constexpr (REGA) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    Areg[tap][kk][m] = *(const uint4*)(wts + tap * COT * 128 + swz(arow + m * 16, kk * 4 + q));
    }
    for (int r = 0; r < reps; ++r) {
        uint4 A0[MT], B0[NT], A1[MT], B1[NT];
        auto load = [&](int tap, int kk, uint4 (&A)[MT], uint4 (&Bf)[NT]) {
            const int kh = tap / 3, kw = tap - kh * 3, chunk = kk * 4 + q;
            if constexpr (!REGA) {
#pragma unroll
                for (int m = 0; m < MT; ++m) A[m] = *(const uint4*)(wts + tap * COT * 128 + swz(arow + m * 16, chunk));
            }
            const char* hb = halo + hcol(c16 + kw, chunk) + (wr * NT + kh) * (HALO * 128);
#pragma unroll
            for (int n = 0; n < NT; ++n) Bf[n] = *(const uint4*)(hb + n * (HALO * 128));
        };
        auto run = [&](int tap, int kk, const uint4 (&A)[MT], const uint4 (&Bf)[NT]) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n) mma(acc[m][n], REGA ? Areg[REGA ? tap : 0][kk][m] : A[m], Bf[n]);
        };
        load(0, 0, A0, B0);
        if constexpr (REGA) {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                load(tap, 1, A1, B1);
                __builtin_amdgcn_sched_barrier(0);
                run(tap, 0, A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                load(tap == 8 ? 0 : tap + 1, 0, A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                run(tap, 1, A1, B1);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll 1
            for (int tap = 0; tap < 9; ++tap) {
                load(tap, 1, A1, B1);
                __builtin_amdgcn_sched_barrier(0);
                run(tap, 0, A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                load(tap == 8 ? 0 : tap + 1, 0, A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                run(tap, 1, A1, B1);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    float s = 0;
    for (int m = 0; m < MT; ++m)
        for (int n = 0; n < NT; ++n) s += acc[m][n][0] + acc[m][n][1] + acc[m][n][2] + acc[m][n][3];
    out[blockIdx.x * blockDim.x + tid] = s;
}

template <int WR, int WC, bool REGA>
void run(const char* name, int ncu, float* out) {
    const int reps = 200;
    const size_t lds = 9 * 64 * 128 + HALO * HALO * 128;
    hipFuncSetAttribute((const void*)k_loop<WR, WC, REGA>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((k_loop<WR, WC, REGA>), dim3(ncu), dim3(64 * WR * WC), lds, 0, out, reps);
    hipEventRecord(e0);
    const int N = 10;
    for (int it = 0; it < N; ++it) hipLaunchKernelGGL((k_loop<WR, WC, REGA>), dim3(ncu), dim3(64 * WR * WC), lds, 0, out, reps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 256 * 64 * 576 * reps * (double)ncu * N;   // one 16x16-px x 64-co tile per rep
    const double us_per_tile = ms * 1e3 / N / reps;
    printf("%-28s %8.3f us/tile  %7.1f TFLOP/s  (ideal tile @2.4GHz 1.92 us)\n", name, us_per_tile, flop / (ms * 1e-3) / 1e12);
}


// 4 waves (one per SIMD), wave tile 64 co x 64 px, fragments read TWO steps ahead
// (three register sets, 18 steps = 9 taps x 2 k-halves, fully unrolled).
template <int GROUPS>
__global__ __launch_bounds__(256 * GROUPS, 1) void k_loop3(float* out, int reps) {
    constexpr int COT = 64, MT = 4, NT = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wts = smem;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    char* halo = smem + 9 * COT * 128 + (wave >> 2) * HALO * HALO * 128;
    const int wr = wave & 3, q = lane >> 4, c16 = lane & 15;
    for (int i = tid; i < (9 * COT * 128 + GROUPS * HALO * HALO * 128) / 4; i += blockDim.x)
        ((unsigned*)smem)[i] = 0x3c003c00u ^ (i * 2654435761u & 0x00ff00ffu);
    __syncthreads();
    f32x4 acc[MT][NT];
    for (int m = 0; m < MT; ++m)
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        uint4 A[3][MT], Bf[3][NT];
        auto load = [&](int st, int buf) {
            const int tap = st >> 1, kk = st & 1;
            const int kh = tap / 3, kw = tap - kh * 3, chunk = kk * 4 + q;
#pragma unroll
            for (int m = 0; m < MT; ++m) A[buf][m] = *(const uint4*)(wts + tap * COT * 128 + swz(m * 16 + c16, chunk));
            const char* hb = halo + hcol(c16 + kw, chunk) + (wr * NT + kh) * (HALO * 128);
#pragma unroll
            for (int n = 0; n < NT; ++n) Bf[buf][n] = *(const uint4*)(hb + n * (HALO * 128));
        };
        load(0, 0);
        load(1, 1);
#pragma unroll
        for (int st = 0; st < 18; ++st) {
            if (st + 2 < 18) load(st + 2, (st + 2) % 3);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n) mma(acc[m][n], A[st % 3][m], Bf[st % 3][n]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float s = 0;
    for (int m = 0; m < MT; ++m)
        for (int n = 0; n < NT; ++n) s += acc[m][n][0] + acc[m][n][1] + acc[m][n][2] + acc[m][n][3];
    out[blockIdx.x * blockDim.x + tid] = s;
}

template <int GROUPS>
void run3(const char* name, int ncu, float* out, int nblk_per_cu) {
    const int reps = 200;
    const size_t lds = 9 * 64 * 128 + GROUPS * HALO * HALO * 128;
    (void)hipFuncSetAttribute((const void*)k_loop3<GROUPS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k_loop3<GROUPS>, dim3(ncu * nblk_per_cu), dim3(256 * GROUPS), lds, 0, out, reps);
    (void)hipEventRecord(e0);
    const int N = 10;
    for (int it = 0; it < N; ++it) hipLaunchKernelGGL(k_loop3<GROUPS>, dim3(ncu * nblk_per_cu), dim3(256 * GROUPS), lds, 0, out, reps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 256 * 64 * 576 * reps * (double)ncu * nblk_per_cu * GROUPS * N;
    printf("%-28s %8.3f us/tile  %7.1f TFLOP/s\n", name, ms * 1e3 / N / reps / nblk_per_cu / GROUPS, flop / (ms * 1e-3) / 1e12);
}


// halo-row reuse order (the production loop): per (kw, k-half) group read NT+2 halo rows
// once and use them for the 3 kh taps.  GROUPS independent wave-groups (own halo each),
// each WR x WC waves, wave tile (64/WC) co x (16/WR rows).
template <int WR, int WC, int GROUPS>
__global__ __launch_bounds__(64 * WR * WC * GROUPS, 1) void k_rows(float* out, int reps) {
    constexpr int COT = 64, MT = COT / 16 / WC, NT = 16 / WR, NB = NT + 2, NWG = WR * WC;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wts = smem;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave / NWG, wig = wave % NWG;
    char* halo = smem + 9 * COT * 128 + grp * HALO * HALO * 128;
    const int wr = wig % WR, wc = wig / WR, q = lane >> 4, c16 = lane & 15;
    for (int i = tid; i < (9 * COT * 128 + GROUPS * HALO * HALO * 128) / 4; i += blockDim.x)
        ((unsigned*)smem)[i] = 0x3c003c00u ^ (i * 2654435761u & 0x00ff00ffu);
    __syncthreads();
    f32x4 acc[MT][NT];
    for (int m = 0; m < MT; ++m)
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0, 0, 0, 0};
    const int arow = wc * MT * 16 + c16;
    for (int r = 0; r < reps; ++r) {
        uint4 A0[3][MT], B0[NB], A1[3][MT], B1[NB];
        auto load = [&](int g, uint4 (&A)[3][MT], uint4 (&Bf)[NB]) {
            const int kw = g >> 1, kk = g & 1, chunk = kk * 4 + q;
            const char* hb = halo + hcol(c16 + kw, chunk) + (wr * NT) * (HALO * 128);
#pragma unroll
            for (int n = 0; n < NB; ++n) Bf[n] = *(const uint4*)(hb + n * (HALO * 128));
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    A[kh][m] = *(const uint4*)(wts + (kh * 3 + kw) * COT * 128 + swz(arow + m * 16, chunk));
        };
        auto run = [&](const uint4 (&A)[3][MT], const uint4 (&Bf)[NB]) {
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int n = 0; n < NT; ++n) mma(acc[m][n], A[kh][m], Bf[n + kh]);
        };
        load(0, A0, B0);
#pragma unroll
        for (int g = 0; g < 6; g += 2) {
            load(g + 1, A1, B1);
            __builtin_amdgcn_sched_barrier(0);
            run(A0, B0);
            __builtin_amdgcn_sched_barrier(0);
            if (g + 2 < 6) load(g + 2, A0, B0);
            __builtin_amdgcn_sched_barrier(0);
            run(A1, B1);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float s = 0;
    for (int m = 0; m < MT; ++m)
        for (int n = 0; n < NT; ++n) s += acc[m][n][0] + acc[m][n][1] + acc[m][n][2] + acc[m][n][3];
    out[blockIdx.x * blockDim.x + tid] = s;
}

template <int WR, int WC, int GROUPS>
void run_rows(const char* name, int ncu, float* out) {
    const int reps = 200;
    const size_t lds = 9 * 64 * 128 + GROUPS * HALO * HALO * 128;
    (void)hipFuncSetAttribute((const void*)k_rows<WR, WC, GROUPS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int T = 64 * WR * WC * GROUPS;
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((k_rows<WR, WC, GROUPS>), dim3(ncu), dim3(T), lds, 0, out, reps);
    (void)hipEventRecord(e0);
    const int N = 10;
    for (int it = 0; it < N; ++it) hipLaunchKernelGGL((k_rows<WR, WC, GROUPS>), dim3(ncu), dim3(T), lds, 0, out, reps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 256 * 64 * 576 * reps * (double)ncu * GROUPS * N;
    printf("%-28s %8.3f us/tile  %7.1f TFLOP/s\n", name, ms * 1e3 / N / reps / GROUPS, flop / (ms * 1e-3) / 1e12);
}

int main() {
    int dev = 0, ncu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    float* out;
    hipMalloc(&out, 256 * 1024 * sizeof(float) * 4);
    run<4, 2, false>("8 waves MT2 NT4 (current)", ncu, out);
    run<4, 1, false>("4 waves MT4 NT4", ncu, out);
    run<8, 1, false>("8 waves MT4 NT2", ncu, out);
    run<2, 2, false>("4 waves MT2 NT8", ncu, out);
    run<4, 2, true>("8 waves MT2 NT4 regA", ncu, out);
    run<4, 1, true>("4 waves MT4 NT4 regA", ncu, out);
    run3<1>("4 waves MT4 NT4 prefetch2", ncu, out, 1);
    run3<2>("2x4 waves MT4 NT4 prefetch2", ncu, out, 1);
    run_rows<4, 2, 1>("rows 8 waves MT2 NT4", ncu, out);
    run_rows<4, 1, 1>("rows 4 waves MT4 NT4", ncu, out);
    run_rows<4, 1, 2>("rows 2x4 waves MT4 NT4", ncu, out);
    run_rows<2, 2, 1>("rows 4 waves MT2 NT8", ncu, out);
    run_rows<2, 2, 2>("rows 2x4 waves MT2 NT8", ncu, out);
    run_rows<4, 2, 2>("rows 2x8 waves MT2 NT4", ncu, out);
    hipFree(out);
    return 0;
}

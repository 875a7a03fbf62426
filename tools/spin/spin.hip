// Diagnostic only (tools/dp_overlap.py): a CU-occupancy stand-in for an RCCL ring all-reduce
// kernel -- `blocks` workgroups of 256 threads, each holding its CU slot for `us` microseconds
// (s_memrealtime, 100 MHz) while touching nothing.  Not part of the product library.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void k_spin(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

extern "C" int spin_launch(int blocks, float us, void* stream) {
    const unsigned long long ticks = (unsigned long long)(us * 100.0f);   // 100 MHz wall clock
    hipLaunchKernelGGL(k_spin, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ticks);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

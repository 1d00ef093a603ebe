// Dev experiment: field-multiply throughput vs instruction-level parallelism (not in the library).
//   mode 0: 2 independent chains, one product per asm column statement (library form)
//   mode 1: 2 chains as one interleaved dual product (mul2_col)
//   mode 2: 4 chains, library form
//   mode 3: 4 chains as two dual products
#include "ecdsa_lane.h"
#include "fe_asm.h"
#include "fe_asm_gen.h"
#include "fe_dual_gen.h"
#include "gpu_common.h"

using namespace bcc;

__device__ __forceinline__ void mul1(fe& r, const fe& a, const fe& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    u32 t[16];
    mul_256x256_col(t, a.v, b.v);
    fe_reduce512_asm(r.v, t);
#endif
}
__device__ __forceinline__ void mul2(fe& r, const fe& a, const fe& b, fe& s, const fe& c, const fe& d) {
#if defined(__HIP_DEVICE_COMPILE__)
    u32 t[16], u[16];
    mul2_col(t, a.v, b.v, u, c.v, d.v);
    fe_reduce512_asm(r.v, t);
    fe_reduce512_asm(s.v, u);
#endif
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_ilp(fe* io, int iters) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    fe a = io[4 * g], b = io[4 * g + 1], c = io[4 * g + 2], d = io[4 * g + 3];
    for (int i = 0; i < iters; i++) {
        if (MODE == 0) { mul1(a, a, b); mul1(c, c, b); }
        if (MODE == 1) { mul2(a, a, b, c, c, b); }
        if (MODE == 2) { mul1(a, a, b); mul1(c, c, b); mul1(d, d, b); mul1(b, b, a); }
        if (MODE == 3) { mul2(a, a, b, c, c, b); mul2(d, d, b, b, b, a); }
    }
    fe_normalize(a); fe_normalize(b); fe_normalize(c); fe_normalize(d);
    io[4 * g] = a; io[4 * g + 1] = b; io[4 * g + 2] = c; io[4 * g + 3] = d;
}

extern "C" int fe_ilp(int mode, int iters, const void* in, void* out, int nblocks, double* ops_per_s) {
    size_t lanes = (size_t)nblocks * 256, bytes = lanes * 4 * sizeof(fe);
    fe* d;
    BCC_HIP_TRY(hipMalloc(&d, bytes));
    BCC_HIP_TRY(hipMemcpy(d, in, bytes, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    BCC_HIP_TRY(hipEventCreate(&e0));
    BCC_HIP_TRY(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; rep++) {
        BCC_HIP_TRY(hipMemcpy(d, in, bytes, hipMemcpyHostToDevice));
        BCC_HIP_TRY(hipEventRecord(e0, 0));
        if (mode == 0) hipLaunchKernelGGL(k_ilp<0>, dim3(nblocks), dim3(256), 0, 0, d, iters);
        if (mode == 1) hipLaunchKernelGGL(k_ilp<1>, dim3(nblocks), dim3(256), 0, 0, d, iters);
        if (mode == 2) hipLaunchKernelGGL(k_ilp<2>, dim3(nblocks), dim3(256), 0, 0, d, iters);
        if (mode == 3) hipLaunchKernelGGL(k_ilp<3>, dim3(nblocks), dim3(256), 0, 0, d, iters);
        BCC_HIP_TRY(hipEventRecord(e1, 0));
        BCC_HIP_TRY(hipEventSynchronize(e1));
    }
    float ms;
    BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    *ops_per_s = (double)lanes * iters * (mode >= 2 ? 4 : 2) / (ms * 1e-3);
    BCC_HIP_TRY(hipMemcpy(out, d, bytes, hipMemcpyDeviceToHost));
    BCC_HIP_TRY(hipFree(d));
    return 0;
}

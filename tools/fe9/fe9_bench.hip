// Dev tool (not part of the library): radix-2^29 (fe29.h) vs radix-2^32 (secp256k1_device.h)
// group-law throughput and cross-check on the GPU.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DBCC_FE9_CHAIN=N -I rust-bitcoinconsensus_amd/csrc -I tools/fe9 \
//         tools/fe9/fe9_bench.hip -o tools/_build/fe9_bench_N.so
// Each lane runs `iters` doublings (op 0/1) or additions (op 2/3) on its own point; occupancy is
// pinned to 4 waves per SIMD like the ladder kernel.
#include "fe29.h"
#include "gpu_common.h"

using namespace bcc;

#define BCC_OCC __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))

__global__ BCC_OCC void k_dbl9(fe* io, int iters) {
    fe* p = io + 6 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
    gej9 a;
    fe9_from_fe(a.x, p[0]); fe9_from_fe(a.y, p[1]); fe9_from_fe(a.z, p[2]);
    for (int i = 0; i < iters; i++) { gej9 t; gej9_double(t, a); a = t; }
    fe9_to_fe(p[0], a.x); fe9_to_fe(p[1], a.y); fe9_to_fe(p[2], a.z);
}
__global__ BCC_OCC void k_add9(fe* io, int iters) {
    fe* p = io + 6 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
    gej9 a;
    fe9 bx, by, bz;
    fe9_from_fe(a.x, p[0]); fe9_from_fe(a.y, p[1]); fe9_from_fe(a.z, p[2]);
    fe9_from_fe(bx, p[3]); fe9_from_fe(by, p[4]); fe9_from_fe(bz, p[5]);
    for (int i = 0; i < iters; i++) { gej9 t; bool inf; gej9_add_zinv(t, inf, a, bx, by, bz, true); a = t; if (inf) break; }
    fe9_to_fe(p[0], a.x); fe9_to_fe(p[1], a.y); fe9_to_fe(p[2], a.z);
}
// the radix-2^32 kernels exactly as the original ISA-count probe (normalised by the host)
__global__ BCC_OCC void k_dbl32(fe* io, int n) {
    fe* p = io + 6 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
    gej a; a.x = p[0]; a.y = p[1]; a.z = p[2];
    for (int i = 0; i < n; i++) { gej t; gej_double(t, a); a = t; }
    p[0] = a.x; p[1] = a.y; p[2] = a.z;
}
__global__ BCC_OCC void k_add32(fe* io, int n) {
    fe* p = io + 6 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
    gej a; a.x = p[0]; a.y = p[1]; a.z = p[2];
    fe bx = p[3], by = p[4], bz = p[5];
    for (int i = 0; i < n; i++) { gej t; bool inf; gej_add_zinv(t, inf, a, bx, by, bz, true); a = t; if (inf) break; }
    p[0] = a.x; p[1] = a.y; p[2] = a.z;
}

extern "C" int fe9_bench(int op, int iters, void* host_io, int nblocks, double* ops_per_s) {
    const size_t lanes = (size_t)nblocks * 256, bytes = lanes * 6 * sizeof(fe);
    fe* d;
    BCC_HIP_TRY(hipMalloc(&d, bytes));
    BCC_HIP_TRY(hipMemcpy(d, host_io, bytes, hipMemcpyHostToDevice));
    auto launch = [&](int it) {
        switch (op) {
            case 0: hipLaunchKernelGGL(k_dbl9, dim3(nblocks), dim3(256), 0, 0, d, it); break;
            case 1: hipLaunchKernelGGL(k_dbl32, dim3(nblocks), dim3(256), 0, 0, d, it); break;
            case 2: hipLaunchKernelGGL(k_add9, dim3(nblocks), dim3(256), 0, 0, d, it); break;
            default: hipLaunchKernelGGL(k_add32, dim3(nblocks), dim3(256), 0, 0, d, it); break;
        }
    };
    hipEvent_t e0, e1;
    BCC_HIP_TRY(hipEventCreate(&e0));
    BCC_HIP_TRY(hipEventCreate(&e1));
    BCC_HIP_TRY(hipEventRecord(e0, 0));
    launch(iters);
    BCC_HIP_TRY(hipEventRecord(e1, 0));
    BCC_HIP_TRY(hipEventSynchronize(e1));
    float ms;
    BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    *ops_per_s = (double)lanes * iters / (ms * 1e-3);
    BCC_HIP_TRY(hipMemcpy(host_io, d, bytes, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

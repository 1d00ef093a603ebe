// Dev tool: calibrate rocprofv3 FETCH_SIZE for the ladder's access pattern (one dword per lane,
// a wave's 64 lanes contiguous = 256 B per load instruction) against a known byte count.
//   hipcc --offload-arch=gfx950 -O3 tools/calib/fetch_calib.cpp -o tools/calib/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -- tools/calib/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read_dwords(const unsigned* __restrict__ buf, unsigned* out, size_t lanes, int W) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= lanes) return;
    const unsigned* p = buf + (t >> 6) * (size_t)(W * 64) + (t & 63);
    unsigned acc = 0;
    for (int w = 0; w < W; w++) acc += p[w * 64];
    out[t] = acc;
}

__global__ void read_x4(const uint4* __restrict__ buf, unsigned* out, size_t lanes, int W) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= lanes) return;
    unsigned acc = 0;
    for (int w = 0; w < W; w++) {
        uint4 v = buf[(size_t)w * lanes + t];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[t] = acc;
}

int main() {
    const size_t lanes = 1 << 20;
    const int W = 192;  // 768 MiB of dwords: beyond L2 and the 256 MiB MALL
    unsigned *buf, *out;
    if (hipMalloc(&buf, lanes * W * 4) != hipSuccess || hipMalloc(&out, lanes * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, lanes * W * 4);
    hipLaunchKernelGGL(read_dwords, dim3(lanes / 256), dim3(256), 0, 0, buf, out, lanes, W);
    hipLaunchKernelGGL(read_x4, dim3(lanes / 256), dim3(256), 0, 0, (const uint4*)buf, out, lanes, W / 4);
    (void)hipDeviceSynchronize();
    printf("read_dwords: %zu bytes; read_x4: %zu bytes\n", lanes * W * 4, lanes * (W / 4) * 16);
    return 0;
}

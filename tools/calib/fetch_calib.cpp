// Dev tool: calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the ECDSA kernels' access patterns
// against known byte counts: one dword per lane (a wave's 64 lanes contiguous = 256 B per load),
// 16 B per lane streaming, and (round 4) the Q-table pattern of K_keyq -- each lane writes its own
// 1 KiB lane-major table as 16-byte stores, then gathers random 64-byte pieces of it (4 x 16 B).
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

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// K_keyq's table writes: lane t's 1 KiB at t * 1 KiB, 64 x 16-byte stores
__global__ void write_tables(uint4* tab, size_t lanes) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= lanes) return;
    uint4* p = tab + t * 64;
    for (int k = 0; k < 64; k++) p[k] = make_uint4((unsigned)t, k, 1, 2);
}

// K_keyq's gathers: R random 64-byte pieces (entry e of 8, half h of 2) of the lane's own table
__global__ void gather_pieces(const uint4* __restrict__ tab, unsigned* out, size_t lanes, int R) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= lanes) return;
    const uint4* p = tab + t * 64;
    unsigned acc = 0;
    for (int r = 0; r < R; r++) {
        const unsigned h = mix32((unsigned)t * 131u + r);
        const uint4* q = p + (h & 7) * 8 + ((h >> 3) & 1) * 4;
        const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
        acc += a.x ^ b.y ^ c.z ^ d.w;
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
    // the table pattern over 1M lanes (1 GiB of tables: beyond L2 and the MALL, as a 1M-lane chunk)
    uint4* tab;
    const int R = 65;  // the Q ladder's additions per verify
    if (hipMalloc(&tab, lanes * 1024) != hipSuccess) return 1;
    hipLaunchKernelGGL(write_tables, dim3(lanes / 256), dim3(256), 0, 0, tab, lanes);
    hipLaunchKernelGGL(gather_pieces, dim3(lanes / 256), dim3(256), 0, 0, (const uint4*)tab, out, lanes, R);
    (void)hipDeviceSynchronize();
    printf("write_tables: %zu bytes; gather_pieces: %zu bytes\n", lanes * 1024, lanes * (size_t)R * 64);
    return 0;
}

// Dev tool: VALU issue rates and dependent latencies on gfx950 that the field-arithmetic design
// depends on (carry-out SGPR write-after-write effects, 64-bit op latency).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/fe9/ubench2.hip -o tools/fe9/_build/ubench2.so
#include <hip/hip_runtime.h>
#include <stdint.h>


template <int OP>
__global__ __launch_bounds__(256) void k_thr(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x;
    uint64_t acc0 = a, acc1 = a + 1, acc2 = a + 2, acc3 = a + 3, acc4 = a + 4, acc5 = a + 5, acc6 = a + 6, acc7 = a + 7;
    uint32_t x0 = a, x1 = a ^ 1, x2 = a ^ 2, x3 = a ^ 3, x4 = a ^ 4, x5 = a ^ 5, x6 = a ^ 6, x7 = a ^ 7;
    for (int it = 0; it < iters; it++) {
#define C_MAD_SAME asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc0) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc1) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc2) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc3) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc4) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc5) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc6) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc7) : "v"(a), "v"(b) : "s0", "s1");
#define C_MAD_DIST asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc0) : "v"(a), "v"(b) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[2:3], %1, %2, %0" : "+v"(acc1) : "v"(a), "v"(b) : "s2", "s3"); asm volatile("v_mad_u64_u32 %0, s[4:5], %1, %2, %0" : "+v"(acc2) : "v"(a), "v"(b) : "s4", "s5"); asm volatile("v_mad_u64_u32 %0, s[6:7], %1, %2, %0" : "+v"(acc3) : "v"(a), "v"(b) : "s6", "s7"); asm volatile("v_mad_u64_u32 %0, s[8:9], %1, %2, %0" : "+v"(acc4) : "v"(a), "v"(b) : "s8", "s9"); asm volatile("v_mad_u64_u32 %0, s[10:11], %1, %2, %0" : "+v"(acc5) : "v"(a), "v"(b) : "s10", "s11"); asm volatile("v_mad_u64_u32 %0, s[12:13], %1, %2, %0" : "+v"(acc6) : "v"(a), "v"(b) : "s12", "s13"); asm volatile("v_mad_u64_u32 %0, s[14:15], %1, %2, %0" : "+v"(acc7) : "v"(a), "v"(b) : "s14", "s15");
#define C_ADDC_DIST asm volatile("v_addc_co_u32_e64 %0, s[16:17], %0, %1, s[16:17]" : "+v"(x0) : "v"(b) : "s16", "s17"); asm volatile("v_addc_co_u32_e64 %0, s[18:19], %0, %1, s[18:19]" : "+v"(x1) : "v"(b) : "s18", "s19"); asm volatile("v_addc_co_u32_e64 %0, s[20:21], %0, %1, s[20:21]" : "+v"(x2) : "v"(b) : "s20", "s21"); asm volatile("v_addc_co_u32_e64 %0, s[22:23], %0, %1, s[22:23]" : "+v"(x3) : "v"(b) : "s22", "s23"); asm volatile("v_addc_co_u32_e64 %0, s[24:25], %0, %1, s[24:25]" : "+v"(x4) : "v"(b) : "s24", "s25"); asm volatile("v_addc_co_u32_e64 %0, s[26:27], %0, %1, s[26:27]" : "+v"(x5) : "v"(b) : "s26", "s27"); asm volatile("v_addc_co_u32_e64 %0, s[28:29], %0, %1, s[28:29]" : "+v"(x6) : "v"(b) : "s28", "s29"); asm volatile("v_addc_co_u32_e64 %0, s[30:31], %0, %1, s[30:31]" : "+v"(x7) : "v"(b) : "s30", "s31");
#define C_ADDCO_DIST asm volatile("v_add_co_u32_e64 %0, s[16:17], %0, %1" : "+v"(x0) : "v"(b) : "s16", "s17"); asm volatile("v_add_co_u32_e64 %0, s[18:19], %0, %1" : "+v"(x1) : "v"(b) : "s18", "s19"); asm volatile("v_add_co_u32_e64 %0, s[20:21], %0, %1" : "+v"(x2) : "v"(b) : "s20", "s21"); asm volatile("v_add_co_u32_e64 %0, s[22:23], %0, %1" : "+v"(x3) : "v"(b) : "s22", "s23"); asm volatile("v_add_co_u32_e64 %0, s[24:25], %0, %1" : "+v"(x4) : "v"(b) : "s24", "s25"); asm volatile("v_add_co_u32_e64 %0, s[26:27], %0, %1" : "+v"(x5) : "v"(b) : "s26", "s27"); asm volatile("v_add_co_u32_e64 %0, s[28:29], %0, %1" : "+v"(x6) : "v"(b) : "s28", "s29"); asm volatile("v_add_co_u32_e64 %0, s[30:31], %0, %1" : "+v"(x7) : "v"(b) : "s30", "s31");
#define C_AND asm volatile("v_and_b32 %0, %0, %1" : "+v"(x0) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x1) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x2) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x3) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x4) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x5) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x6) : "v"(b)); asm volatile("v_and_b32 %0, %0, %1" : "+v"(x7) : "v"(b));
#define C_MOV asm volatile("v_mov_b32 %0, %1" : "=v"(x0) : "v"(x0 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x1) : "v"(x1 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x2) : "v"(x2 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x3) : "v"(x3 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x4) : "v"(x4 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x5) : "v"(x5 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x6) : "v"(x6 ^ b)); asm volatile("v_mov_b32 %0, %1" : "=v"(x7) : "v"(x7 ^ b));
#define C_SUB asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x0) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x1) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x2) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x3) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x4) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x5) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x6) : "v"(b)); asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x7) : "v"(b));
#define C_LSHL asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x0) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x1) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x2) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x3) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x4) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x5) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x6) : ); asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x7) : );
#define C_ADD3 asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x0) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x1) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x2) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x3) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x4) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x5) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x6) : "v"(b)); asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x7) : "v"(b));
#define C_LSHLADD32 asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x0) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x1) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x2) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x3) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x4) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x5) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x6) : "v"(b)); asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x7) : "v"(b));
#define C_BFE asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x0) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x1) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x2) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x3) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x4) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x5) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x6) : ); asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x7) : );
#define C_SHR64 asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc0) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc1) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc2) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc3) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc4) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc5) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc6) : ); asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc7) : );
#define C_MADADDC asm volatile("v_mad_u64_u32 %0, s[16:17], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[16:17], 0, %1, s[16:17]" : "+v"(acc0), "+v"(x0) : "v"(a), "v"(b) : "s16", "s17"); asm volatile("v_mad_u64_u32 %0, s[18:19], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[18:19], 0, %1, s[18:19]" : "+v"(acc1), "+v"(x1) : "v"(a), "v"(b) : "s18", "s19"); asm volatile("v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[20:21], 0, %1, s[20:21]" : "+v"(acc2), "+v"(x2) : "v"(a), "v"(b) : "s20", "s21"); asm volatile("v_mad_u64_u32 %0, s[22:23], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[22:23], 0, %1, s[22:23]" : "+v"(acc3), "+v"(x3) : "v"(a), "v"(b) : "s22", "s23"); asm volatile("v_mad_u64_u32 %0, s[24:25], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[24:25], 0, %1, s[24:25]" : "+v"(acc4), "+v"(x4) : "v"(a), "v"(b) : "s24", "s25"); asm volatile("v_mad_u64_u32 %0, s[26:27], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[26:27], 0, %1, s[26:27]" : "+v"(acc5), "+v"(x5) : "v"(a), "v"(b) : "s26", "s27"); asm volatile("v_mad_u64_u32 %0, s[28:29], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[28:29], 0, %1, s[28:29]" : "+v"(acc6), "+v"(x6) : "v"(a), "v"(b) : "s28", "s29"); asm volatile("v_mad_u64_u32 %0, s[30:31], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[30:31], 0, %1, s[30:31]" : "+v"(acc7), "+v"(x7) : "v"(a), "v"(b) : "s30", "s31");
        if (OP == 0) { C_MAD_SAME }
        if (OP == 1) { C_MAD_DIST }
        if (OP == 2) { C_ADDC_DIST }
        if (OP == 3) { C_ADDCO_DIST }
        if (OP == 4) { C_AND }
        if (OP == 5) { C_MOV }
        if (OP == 6) { C_SUB }
        if (OP == 7) { C_LSHL }
        if (OP == 8) { C_ADD3 }
        if (OP == 9) { C_LSHLADD32 }
        if (OP == 10) { C_BFE }
        if (OP == 11) { C_SHR64 }
        if (OP == 12) { C_MADADDC }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(acc0 ^ acc1 ^ acc2 ^ acc3 ^ acc4 ^ acc5 ^ acc6 ^ acc7) ^
                                                 x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}

// dependent-chain latency, one wave per SIMD: cycles per instruction from s_memtime
template <int OP>
__global__ __launch_bounds__(64) void k_lat(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) {
    uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x, x = a;
    uint64_t acc = a;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#define L8(S) S S S S S S S S
        if (OP == 0) { L8(asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "s0", "s1");) }
        if (OP == 1) { L8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));) }
        if (OP == 2) { L8(asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc));) }
        if (OP == 3) { L8(asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0\n\tv_lshrrev_b64 %0, 29, %0" : "+v"(acc) : "v"(a), "v"(b) : "s0", "s1");) }
        if (OP == 4) { L8(asm volatile("v_add_co_u32_e64 %0, s[0:1], %0, %1\n\tv_addc_co_u32_e64 %0, s[0:1], %0, %1, s[0:1]" : "+v"(x) : "v"(b) : "s0", "s1");) }
        if (OP == 5) { L8(asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));) }
        if (OP == 6) {  // 8 independent adds: the issue cost of a lone wave (calibration)
            asm volatile("v_add_u32 %0, %0, %1\n\tv_add_u32 %2, %2, %1\n\tv_add_u32 %3, %3, %1\n\tv_add_u32 %4, %4, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %2, %2, %1\n\tv_add_u32 %3, %3, %1\n\tv_add_u32 %4, %4, %1"
                         : "+v"(x), "+v"(b), "+v"(a), "+v"(seed) : "v"(b));
        }
        if (OP == 7) {  // 8 independent mads (distinct carry SGPRs): lone-wave issue cost
            uint64_t q1 = acc + 1, q2 = acc + 2, q3 = acc + 3;
            asm volatile("v_mad_u64_u32 %0, s[0:1], %4, %5, %0\n\tv_mad_u64_u32 %1, s[2:3], %4, %5, %1\n\tv_mad_u64_u32 %2, s[4:5], %4, %5, %2\n\tv_mad_u64_u32 %3, s[6:7], %4, %5, %3\n\tv_mad_u64_u32 %0, s[0:1], %4, %5, %0\n\tv_mad_u64_u32 %1, s[2:3], %4, %5, %1\n\tv_mad_u64_u32 %2, s[4:5], %4, %5, %2\n\tv_mad_u64_u32 %3, s[6:7], %4, %5, %3"
                         : "+v"(acc), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(a), "v"(b) : "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7");
            acc ^= q1 ^ q2 ^ q3;
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)acc ^ (uint32_t)(acc >> 32) ^ x;
}

#define LAUNCH_T(K) case K: hipLaunchKernelGGL(k_thr<K>, dim3(grid), dim3(256), 0, 0, out, it, 1u); break;
#define LAUNCH_L(K) case K: hipLaunchKernelGGL(k_lat<K>, dim3(grid), dim3(64), 0, 0, out, cyc, it, 1u); break;

extern "C" int ub_throughput(int op, int iters, double* rate) {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 8;
    uint32_t* out;
    if (hipMalloc(&out, (size_t)grid * 256 * 4)) return 1;
    auto go = [&](int it) {
        switch (op) { LAUNCH_T(0) LAUNCH_T(1) LAUNCH_T(2) LAUNCH_T(3) LAUNCH_T(4) LAUNCH_T(5) LAUNCH_T(6)
                      LAUNCH_T(7) LAUNCH_T(8) LAUNCH_T(9) LAUNCH_T(10) LAUNCH_T(11) LAUNCH_T(12) }
    };
    go(16);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    go(iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const int per = op == 12 ? 16 : 8;
    *rate = (double)grid * 256 * iters * per / (ms * 1e-3);
    hipFree(out);
    return 0;
}

extern "C" int ub_latency(int op, int iters, double* cycles_per_instr) {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 4;  // one wave per SIMD
    uint32_t* out;
    uint64_t* cyc;
    if (hipMalloc(&out, (size_t)grid * 64 * 4) || hipMalloc(&cyc, grid * 8)) return 1;
    auto go = [&](int it) { switch (op) { LAUNCH_L(0) LAUNCH_L(1) LAUNCH_L(2) LAUNCH_L(3) LAUNCH_L(4) LAUNCH_L(5) LAUNCH_L(6) LAUNCH_L(7) } };
    go(16);
    go(iters);
    hipDeviceSynchronize();
    uint64_t h[4096];
    hipMemcpy(h, cyc, 8 * (grid < 4096 ? grid : 4096), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid && i < 4096; i++) s += (double)h[i];
    const int per = (op == 3 || op == 4) ? 16 : 8;
    // s_memtime counts at the shader clock on gfx950? reported raw: ticks per instruction
    *cycles_per_instr = s / (grid < 4096 ? grid : 4096) / ((double)iters * per);
    hipFree(out);
    hipFree(cyc);
    return 0;
}

// Hot-path stage (a) on gfx950: SHA-256d over host-padded messages, one lane per message.
//   K1 sha256d_msgs   aux messages (BIP143 hashPrevouts / hashSequence / hashOutputs) -> 32 B
//   K2 patch_digests  scatter aux digests into the BIP143 preimage slots
//   K3 sha256d_msgs   preimages -> sighash, written straight into the ECDSA tuple msg rows
// Integer-ALU bound (~2k VALU ops per 64-byte block); HBM traffic per launch is reported by
// bench.py as the algorithmic bytes (message bytes in + 32 B out per message).
#include <chrono>
#include <memory>

#include "gpu_common.h"
#include "pipeline.h"
#include "sha256_device.h"

namespace bcc {

__device__ __forceinline__ uint32_t bswap_u32(uint32_t x) { return __builtin_bswap32(x); }

// Each lane streams its own message 64 bytes at a time (four 16-byte loads; messages are
// 64-byte aligned so every load is a full aligned 16-byte access).
__device__ __forceinline__ void sha256d_msg_lane(const uint8_t* __restrict__ buf,
                                                 const uint32_t* __restrict__ off_blk,
                                                 const uint32_t* __restrict__ nblk, uint32_t m,
                                                 uint8_t* __restrict__ out,
                                                 const uint32_t* __restrict__ out_row) {
    const uint4* p = reinterpret_cast<const uint4*>(buf + (size_t)off_blk[m] * 64);
    uint32_t st[8];
    sha256_init_state(st);
    const uint32_t nb = nblk[m];
    uint4 nxt[4];  // the next block, fetched while the current one is compressed
#pragma unroll
    for (int q = 0; q < 4; q++) nxt[q] = p[q];
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            w[4 * q + 0] = bswap_u32(nxt[q].x);
            w[4 * q + 1] = bswap_u32(nxt[q].y);
            w[4 * q + 2] = bswap_u32(nxt[q].z);
            w[4 * q + 3] = bswap_u32(nxt[q].w);
        }
        if (b + 1 < nb) {
#pragma unroll
            for (int q = 0; q < 4; q++) nxt[q] = p[(b + 1) * 4 + q];
        }
        sha256_compress(st, w);
    }
    uint32_t d[8];
    sha256_of_digest(d, st);
    uint32_t row = out_row ? out_row[m] : m;
    uint4* o = reinterpret_cast<uint4*>(out + (size_t)row * 32);
    o[0] = make_uint4(bswap_u32(d[0]), bswap_u32(d[1]), bswap_u32(d[2]), bswap_u32(d[3]));
    o[1] = make_uint4(bswap_u32(d[4]), bswap_u32(d[5]), bswap_u32(d[6]), bswap_u32(d[7]));
}

__global__ __launch_bounds__(256) void sha256d_msgs_kernel(const uint8_t* __restrict__ buf,
                                                           const uint32_t* __restrict__ off_blk,
                                                           const uint32_t* __restrict__ nblk,
                                                           uint32_t nmsg, uint8_t* __restrict__ out,
                                                           const uint32_t* __restrict__ out_row) {
    uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m < nmsg) sha256d_msg_lane(buf, off_blk, nblk, m, out, out_row);
}

// K3': legacy SIGHASH_ALL preimages assembled from the tx template while hashing (TplJob).
// Message byte g: T[g] (g < pos), code[g - pos] (< pos + code_len), T[g - code_len + 1]
// (< L - 4), le32(hashtype), then SHA padding.  Whole words inside the first / third segment
// come from aligned dword loads (the third with a funnel shift); only the few words that
// straddle a segment boundary or the padding are assembled byte by byte.  The next block's words
// are fetched before the current block is compressed, so a long (many-input) message does not
// pay one load latency per block.  Wave-sized workgroups: the long jobs of one big tx spread over
// many CUs.
struct TplMsg {
    const uint8_t* T;
    const uint8_t* C;
    uint32_t pos, s3, e3, L, tail, ht;
};

__device__ __forceinline__ uint32_t tpl_byte(const TplMsg& m, uint32_t g) {
    if (g < m.pos) return m.T[g];
    if (g < m.s3) return m.C[g - m.pos];
    if (g < m.e3) return m.T[g - (m.s3 - m.pos) + 1];
    if (g < m.L) return (m.ht >> (8 * (g - m.e3))) & 0xffu;
    if (g == m.L) return 0x80u;
    if (g >= m.tail) {  // 64-bit big-endian bit length
        uint64_t bits = (uint64_t)m.L * 8;
        return (uint32_t)(bits >> (8 * (7 - (g - m.tail)))) & 0xffu;
    }
    return 0u;
}

__device__ __forceinline__ uint32_t tpl_word(const TplMsg& m, uint32_t q) {
    if (q + 4 <= m.pos) return bswap_u32(*reinterpret_cast<const uint32_t*>(m.T + q));
    if (q >= m.s3 && q + 4 <= m.e3) {
        uint32_t o = q - (m.s3 - m.pos) + 1;
        const uint32_t* a = reinterpret_cast<const uint32_t*>(m.T + (o & ~3u));
        return bswap_u32(__builtin_amdgcn_alignbyte(a[1], a[0], o & 3u));
    }
    if (q > m.L && q + 4 <= m.tail) return 0u;
    return (tpl_byte(m, q) << 24) | (tpl_byte(m, q + 1) << 16) | (tpl_byte(m, q + 2) << 8) |
           tpl_byte(m, q + 3);
}

__device__ __forceinline__ void sha256d_tpl_lane(const uint8_t* __restrict__ tpl,
                                                 const uint8_t* __restrict__ code,
                                                 const TplJob* __restrict__ jobs, uint32_t i,
                                                 uint8_t* __restrict__ out) {
    const TplJob j = jobs[i];
    TplMsg m;
    m.T = tpl + j.tpl_off;
    m.C = code + j.code_off;
    m.pos = j.pos;
    m.s3 = j.pos + j.code_len;
    m.L = j.tpl_len - 1 + j.code_len + 4;
    m.e3 = m.L - 4;
    m.tail = j.nblk * 64 - 8;
    m.ht = j.hashtype;
    uint32_t st[8];
    sha256_init_state(st);
    uint32_t nxt[16];
#pragma unroll
    for (int w = 0; w < 16; w++) nxt[w] = tpl_word(m, 4 * w);
    for (uint32_t b = 0; b < j.nblk; b++) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = nxt[k];
        if (b + 1 < j.nblk) {
#pragma unroll
            for (int k = 0; k < 16; k++) nxt[k] = tpl_word(m, 64 * (b + 1) + 4 * k);
        }
        sha256_compress(st, w);
    }
    uint32_t d[8];
    sha256_of_digest(d, st);
    uint4* o = reinterpret_cast<uint4*>(out + (size_t)j.row * 32);
    o[0] = make_uint4(bswap_u32(d[0]), bswap_u32(d[1]), bswap_u32(d[2]), bswap_u32(d[3]));
    o[1] = make_uint4(bswap_u32(d[4]), bswap_u32(d[5]), bswap_u32(d[6]), bswap_u32(d[7]));
}

// K1 + K3' fused: lanes [0, naux) hash the aux messages, lanes [naux, naux + ntpl) the template
// jobs.  Neither depends on the other, so one launch overlaps the two longest serial chains of a
// many-input tx (its hashPrevouts message and its legacy preimages) instead of running them back
// to back.
__global__ __launch_bounds__(64) void sha256d_aux_tpl_kernel(
    const uint8_t* __restrict__ aux, const uint32_t* __restrict__ aux_off,
    const uint32_t* __restrict__ aux_nblk, uint32_t naux, uint8_t* __restrict__ auxd,
    const uint8_t* __restrict__ tpl, const uint8_t* __restrict__ code,
    const TplJob* __restrict__ jobs, uint32_t ntpl, uint8_t* __restrict__ msg) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < naux)
        sha256d_msg_lane(aux, aux_off, aux_nblk, i, auxd, nullptr);
    else if (i - naux < ntpl)
        sha256d_tpl_lane(tpl, code, jobs, i - naux, msg);
}


__global__ __launch_bounds__(256) void patch_digests_kernel(uint8_t* __restrict__ pre,
                                                            const PatchRec* __restrict__ patches,
                                                            const uint8_t* __restrict__ auxd,
                                                            uint32_t npatch) {
    // one lane per patch: the 32-byte digest with the widest stores the slot's alignment allows
    // (BIP143 slots sit at preimage offsets 4, 36 and len - 40)
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npatch) return;
    const PatchRec p = patches[i];
    const uint4* src = reinterpret_cast<const uint4*>(auxd + (size_t)p.aux * 32);
    const uint4 d0 = src[0], d1 = src[1];
    const uint32_t w[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
    uint8_t* dst = pre + p.pre_byte;
    if ((p.pre_byte & 3) == 0) {
        uint32_t* o = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = w[k];
    } else if ((p.pre_byte & 1) == 0) {
        uint16_t* o = reinterpret_cast<uint16_t*>(dst);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            o[2 * k] = (uint16_t)w[k];
            o[2 * k + 1] = (uint16_t)(w[k] >> 16);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 32; k++) dst[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
}

// ------------------------------------------------------------------------------------------
DeviceBatch::DeviceBatch(int device) : dev_(device) {}

DeviceBatch::~DeviceBatch() {
    (void)hipSetDevice(dev_);
    if (own_stream_) (void)hipStreamDestroy((hipStream_t)own_stream_);
    if (side_stream_) (void)hipStreamDestroy((hipStream_t)side_stream_);
    if (ev_fork_) (void)hipEventDestroy((hipEvent_t)ev_fork_);
    if (ev_join_) (void)hipEventDestroy((hipEvent_t)ev_join_);
    if (arena_) (void)hipFree(arena_);
}

void* DeviceBatch::pick(void* stream) {
    if (!stream) {
        if (!own_stream_) {
            hipStream_t s = nullptr;
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
            own_stream_ = s;
        }
        stream = own_stream_;
    }
    last_stream_ = stream;
    return stream;
}

int DeviceBatch::sync() {
    BCC_HIP_TRY(hipSetDevice(dev_));
    if (last_stream_) BCC_HIP_TRY(hipStreamSynchronize((hipStream_t)last_stream_));
    return 0;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int DeviceBatch::stage(const SighashJobs& j, const TupleRows& rows) {
    if (int e = sync()) return e;  // the previous run may still read the arena
    n_rows_ = rows.size();
    n_pre_ = j.pre_off.size();
    n_aux_ = j.aux_off.size();
    n_patch_ = j.patches.size();
    pre_blocks_ = j.pre.size() / 64;
    aux_blocks_ = j.aux.size() / 64;
    n_tjob_ = j.tjobs.size();
    tjob_blocks_ = 0;
    for (const auto& t : j.tjobs) tjob_blocks_ += t.nblk;
    const size_t R = n_rows_;
    size_t sizes[] = {R,         32 * R,           32 * R,         32 * R,        32 * R,
                      32 * R,    R,                j.aux.size(),   j.pre.size(),  32 * n_aux_,
                      4 * n_aux_, 4 * n_aux_,      4 * n_pre_,     4 * n_pre_,    4 * n_pre_,
                      sizeof(PatchRec) * n_patch_, j.tpl.size(),   j.code.size(),
                      sizeof(TplJob) * n_tjob_};
    const int NB = sizeof(sizes) / sizeof(sizes[0]);
    size_t total = 0;
    for (int i = 0; i < NB; i++) total += align256(sizes[i]);
    if (total > cap_) {
        if (arena_) BCC_HIP_TRY(hipFree(arena_));
        arena_ = nullptr;
        cap_ = 0;
        BCC_HIP_TRY(hipMalloc(&arena_, total));
        cap_ = total;
    }
    uint8_t* p = (uint8_t*)arena_;
    uint8_t* ptr[NB];
    for (int i = 0; i < NB; i++) {
        ptr[i] = p;
        p += align256(sizes[i]);
    }
    d_tag = ptr[0]; d_x = ptr[1]; d_y = ptr[2]; d_r = ptr[3]; d_s = ptr[4]; d_m = ptr[5];
    d_v = ptr[6]; d_aux_ = ptr[7]; d_pre_ = ptr[8]; d_auxd_ = ptr[9];
    d_aux_off_ = (uint32_t*)ptr[10]; d_aux_nblk_ = (uint32_t*)ptr[11];
    d_pre_off_ = (uint32_t*)ptr[12]; d_pre_nblk_ = (uint32_t*)ptr[13];
    d_pre_row_ = (uint32_t*)ptr[14]; d_patch_ = (PatchRec*)ptr[15];
    d_tpl_ = ptr[16]; d_code_ = ptr[17]; d_tjob_ = (TplJob*)ptr[18];
    const void* src[] = {rows.tag.data(), rows.x.data(), rows.y.data(), rows.r.data(),
                         rows.s.data(), rows.msg.data(), nullptr, j.aux.data(), j.pre.data(),
                         nullptr, j.aux_off.data(), j.aux_nblk.data(), j.pre_off.data(),
                         j.pre_nblk.data(), j.pre_row.data(), j.patches.data(), j.tpl.data(),
                         j.code.data(), j.tjobs.data()};
    for (int i = 0; i < NB; i++)
        if (src[i] && sizes[i]) BCC_HIP_TRY(hipMemcpy(ptr[i], src[i], sizes[i], hipMemcpyHostToDevice));
    return 0;
}

int DeviceBatch::run_sighash(void* stream) {
    BCC_HIP_TRY(hipSetDevice(dev_));
    hipStream_t st = (hipStream_t)pick(stream);
    if (!st) return (int)hipErrorOutOfMemory;
    if (n_aux_ + n_tjob_) {  // K1 + K3' in one launch
        const size_t lanes = n_aux_ + n_tjob_;
        hipLaunchKernelGGL(sha256d_aux_tpl_kernel, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, st,
                           d_aux_, d_aux_off_, d_aux_nblk_, (uint32_t)n_aux_, d_auxd_, d_tpl_, d_code_,
                           d_tjob_, (uint32_t)n_tjob_, d_m);
        BCC_HIP_TRY(hipGetLastError());
    }
    if (n_patch_) {
        size_t th = n_patch_;
        hipLaunchKernelGGL(patch_digests_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st,
                           d_pre_, d_patch_, d_auxd_, (uint32_t)n_patch_);
        BCC_HIP_TRY(hipGetLastError());
    }
    if (n_pre_) {
        hipLaunchKernelGGL(sha256d_msgs_kernel, dim3((unsigned)((n_pre_ + 255) / 256)), dim3(256), 0, st,
                           d_pre_, d_pre_off_, d_pre_nblk_, (uint32_t)n_pre_, d_m, d_pre_row_);
        BCC_HIP_TRY(hipGetLastError());
    }
    return 0;
}

int DeviceBatch::run_ecdsa(void* stream) {
    BCC_HIP_TRY(hipSetDevice(dev_));
    void* st = pick(stream);
    if (!st) return (int)hipErrorOutOfMemory;
    return ecdsa_launch(scratch_, d_tag, d_x, d_y, d_r, d_s, d_m, d_v, n_rows_, st);
}

// K_inv and K_key read only the s and key rows, so they run on a side stream beside the sighash
// kernels (fork / join by events: graph-capturable); prep + ladder wait for both.
int DeviceBatch::run(void* stream) {
    BCC_HIP_TRY(hipSetDevice(dev_));
    hipStream_t st = (hipStream_t)pick(stream);
    if (!st) return (int)hipErrorOutOfMemory;
    if (n_rows_ == 0 || n_aux_ + n_tjob_ + n_pre_ == 0) {
        if (int e = run_sighash(st)) return e;
        return run_ecdsa(st);
    }
    if (!side_stream_) {
        hipStream_t s = nullptr;
        hipEvent_t a = nullptr, b = nullptr;
        BCC_HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        BCC_HIP_TRY(hipEventCreateWithFlags(&a, hipEventDisableTiming));
        BCC_HIP_TRY(hipEventCreateWithFlags(&b, hipEventDisableTiming));
        side_stream_ = s;
        ev_fork_ = a;
        ev_join_ = b;
    }
    hipStream_t side = (hipStream_t)side_stream_;
    BCC_HIP_TRY(hipEventRecord((hipEvent_t)ev_fork_, st));
    BCC_HIP_TRY(hipStreamWaitEvent(side, (hipEvent_t)ev_fork_, 0));
    if (int e = ecdsa_launch_pre(scratch_, d_tag, d_x, d_y, d_s, n_rows_, side)) return e;
    BCC_HIP_TRY(hipEventRecord((hipEvent_t)ev_join_, side));
    if (int e = run_sighash(st)) return e;
    BCC_HIP_TRY(hipStreamWaitEvent(st, (hipEvent_t)ev_join_, 0));
    return ecdsa_launch_after_pre(scratch_, d_x, d_r, d_s, d_m, d_v, n_rows_, st);
}

int DeviceBatch::fetch_verdicts(uint8_t* out) {
    if (int e = sync()) return e;
    if (n_rows_) BCC_HIP_TRY(hipMemcpy(out, d_v, n_rows_, hipMemcpyDeviceToHost));
    return 0;
}

int DeviceBatch::fetch_msgs(uint8_t* out) {
    if (int e = sync()) return e;
    if (n_rows_) BCC_HIP_TRY(hipMemcpy(out, d_m, 32 * n_rows_, hipMemcpyDeviceToHost));
    return 0;
}

int gpu_verify_batch(int device, const SighashJobs& jobs, const TupleRows& rows, uint8_t* verdict,
                     double* stage_seconds) {
    if (rows.size() == 0) return 0;
    // one cached batch per (thread, device): repeated calls reuse the device arena, scratch and
    // stream, and concurrent callers never share any of them
    thread_local std::vector<std::unique_ptr<DeviceBatch>> cache;
    if (device < 0) return (int)hipErrorInvalidDevice;
    if ((int)cache.size() <= device) cache.resize(device + 1);
    if (!cache[device]) cache[device] = std::make_unique<DeviceBatch>(device);
    DeviceBatch& b = *cache[device];
    auto t0 = std::chrono::steady_clock::now();
    if (int e = b.stage(jobs, rows)) return e;
    if (stage_seconds)
        *stage_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (int e = b.run(nullptr)) return e;
    return b.fetch_verdicts(verdict);
}

}  // namespace bcc

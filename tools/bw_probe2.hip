// bw_probe2.hip — write ceiling for the 4-byte-slot store pattern of
// k_apply_fast: per wave item, R node rows of C consecutive KiB each (rows
// shard_len * 4 B apart), optionally after a dependent metadata load + a
// vmcnt(0) wait per item (what the apply kernel does per bucket).
// Measurement tool, not part of the engine.
//
//   hipcc -O3 --offload-arch=gfx950 tools/bw_probe2.hip -o tools/bw_probe2 && tools/bw_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ inline uint64_t xcd_id(uint32_t wv)
{
    const uint64_t per = (uint64_t)(gridDim.x >> 3) * 4;
    return (uint64_t)(blockIdx.x & 7) * per + (uint64_t)(blockIdx.x >> 3) * 4 + wv;
}

// item = C consecutive 1-KiB buckets; R rows; LOAD: one dependent 16-B load
// per lane from `meta` (two levels) + vmcnt(0) before the item's stores
template <int C, bool LOAD, bool NT = false>
__global__ __launch_bounds__(256) void k_rows(uint32_t *st, const uint64_t *meta, uint64_t NB, uint32_t R,
                                              uint64_t L, unsigned long long *sink)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t items = NB / C;
    uint64_t acc = 0;
    for (uint64_t it = xcd_id(wv); it < items; it += nwaves) {
        uint32_t q = (uint32_t)it;
        if (LOAD) {
            const uint64_t a = meta[(it * 64 + lane) & ((1ull << 24) - 1)];
            const uint64_t b2 = meta[(a + lane) & ((1ull << 24) - 1)];
            __builtin_amdgcn_s_waitcnt(0x0F70);
            q += (uint32_t)b2;
            acc += b2;
        }
        for (uint32_t r = 0; r < R; ++r) {
            uint32_t *row = st + (uint64_t)r * L + it * C * 256;
#pragma unroll
            for (int c = 0; c < C; ++c)
            {
                u32x4 *dst = reinterpret_cast<u32x4 *>(row + c * 256 + 4 * lane);
                const u32x4 val = u32x4{q, q + 1, q + 2, q + r};
                if (NT) __builtin_nontemporal_store(val, dst);
                else *dst = val;
            }
        }
    }
    if (acc == 0x123456789ull) *sink = acc;
}

template <int C, bool LOAD, bool NT = false>
static void run(const char *name, uint32_t *st, const uint64_t *meta, uint64_t NB, uint32_t R, uint64_t L,
                unsigned long long *sink, int cus)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int wpc : {4, 8, 16}) {
        const uint32_t grid = cus * wpc;
        float best = 1e9f;
        for (int r = 0; r < 4; ++r) {
            hipEventRecord(a);
            hipLaunchKernelGGL((k_rows<C, LOAD, NT>), dim3(grid), dim3(256), 0, 0, st, meta, NB, R, L, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (r && ms < best) best = ms;
        }
        const double bytes = (double)R * L * 4;
        printf("%-28s wgs/cu %2d: %.3f ms  %.2f TB/s\n", name, wpc, best, bytes / (best * 1e-3) / 1e12);
    }
    hipEventDestroy(a); hipEventDestroy(b);
}

int main()
{
    const uint32_t R = 10;
    const uint64_t L = 1ull << 27, NB = L >> 8;
    uint32_t *st = nullptr;
    uint64_t *meta = nullptr;
    unsigned long long *sink = nullptr;
    if (hipMalloc(&st, (size_t)R * L * 4) != hipSuccess || hipMalloc(&meta, 8ull << 24) != hipSuccess ||
        hipMalloc(&sink, 8) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(meta, 0, 8ull << 24);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<1, false>("1 KiB/row, no load", st, meta, NB, R, L, sink, cus);
    run<2, false>("2 KiB/row, no load", st, meta, NB, R, L, sink, cus);
    run<4, false>("4 KiB/row, no load", st, meta, NB, R, L, sink, cus);
    run<1, true>("1 KiB/row, load+wait", st, meta, NB, R, L, sink, cus);
    run<2, true>("2 KiB/row, load+wait", st, meta, NB, R, L, sink, cus);
    run<4, true>("4 KiB/row, load+wait", st, meta, NB, R, L, sink, cus);
    run<1, false, true>("1 KiB/row, no load, nt", st, meta, NB, R, L, sink, cus);
    run<4, false, true>("4 KiB/row, no load, nt", st, meta, NB, R, L, sink, cus);
    run<1, true, true>("1 KiB/row, load+wait, nt", st, meta, NB, R, L, sink, cus);
    run<4, true, true>("4 KiB/row, load+wait, nt", st, meta, NB, R, L, sink, cus);
    {
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        float best = 1e9f;
        for (int r = 0; r < 4; ++r) {
            hipEventRecord(a);
            hipMemsetD32Async((hipDeviceptr_t)st, r, (size_t)R * L, 0);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (r && ms < best) best = ms;
        }
        printf("%-28s          : %.3f ms  %.2f TB/s\n", "hipMemsetD32", best, (double)R * L * 4 / (best * 1e-3) / 1e12);
    }
    hipFree(st); hipFree(meta); hipFree(sink);
    return 0;
}

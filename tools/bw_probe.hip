// bw_probe.hip — write-bandwidth ceiling for the state-store pattern of
// k_apply_fast (one wave writes a 4 KiB bucket of one node's 16-B slots with
// four 16-B-per-lane stores).  Measurement tool, not part of the engine.
//
//   hipcc -O3 --offload-arch=gfx950 tools/bw_probe.hip -o tools/bw_probe && tools/bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// mode 0: bucket-major (wave: bucket b, nodes 0..N-1), mode 1: node-major sweep
template <bool NT>
__global__ __launch_bounds__(256) void k_write(uint64_t *st, uint64_t NB, uint32_t N, uint64_t L, int mode)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t wid = (uint64_t)blockIdx.x * 4 + wv;
    const uint64_t items = NB * N;
    for (uint64_t it = wid; it < items; it += nwaves) {
        uint64_t b, n;
        if (mode == 0) { b = it / N; n = it % N; } else { n = it / NB; b = it % NB; }
        uint64_t *row = st + 2 * (n * L + (b << 8));
        u64x2 w0 = {it, lane}, w1 = {it + 1, lane}, w2 = {it + 2, lane}, w3 = {it + 3, lane};
        u64x2 *p = reinterpret_cast<u64x2 *>(row);
        if (NT) {
            __builtin_nontemporal_store(w0, p + 2 * lane);
            __builtin_nontemporal_store(w1, p + 2 * lane + 1);
            __builtin_nontemporal_store(w2, p + 128 + 2 * lane);
            __builtin_nontemporal_store(w3, p + 128 + 2 * lane + 1);
        } else {
            p[2 * lane] = w0; p[2 * lane + 1] = w1; p[128 + 2 * lane] = w2; p[128 + 2 * lane + 1] = w3;
        }
    }
}

// plain streaming copy-free write: each lane one 16-B store per iteration, grid-stride
__global__ __launch_bounds__(256) void k_fill(u64x2 *p, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) p[i] = u64x2{i, i};
}

int main()
{
    const uint32_t N = 9;
    const uint64_t L = 1ull << 27, NB = L >> 8;
    const uint64_t bytes = (uint64_t)N * L * 16;
    uint64_t *st = nullptr;
    if (hipMalloc(&st, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int rep = 0; rep < 2; ++rep)
        for (int wpc : {2, 4, 8, 16}) {
            const uint32_t grid = cus * wpc;
            for (int mode = 0; mode < 2; ++mode)
                for (int nt = 0; nt < 2; ++nt) {
                    float best = 1e9f;
                    for (int r = 0; r < 3; ++r) {
                        hipEventRecord(a);
                        if (nt) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, st, NB, N, L, mode);
                        else hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, st, NB, N, L, mode);
                        hipEventRecord(b);
                        hipEventSynchronize(b);
                        float ms = 0;
                        hipEventElapsedTime(&ms, a, b);
                        if (ms < best) best = ms;
                    }
                    if (rep) printf("write wgs/cu %2d %s %s: %.3f ms  %.2f TB/s\n", wpc, mode ? "node-major  " : "bucket-major",
                                    nt ? "nt   " : "plain", best, bytes / (best * 1e-3) / 1e12);
                }
            float best = 1e9f;
            for (int r = 0; r < 3; ++r) {
                hipEventRecord(a);
                hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, 0, reinterpret_cast<u64x2 *>(st), bytes / 16);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            if (rep) printf("fill  wgs/cu %2d: %.3f ms  %.2f TB/s\n", wpc, best, bytes / (best * 1e-3) / 1e12);
        }
    hipFree(st);
    return 0;
}

// fetch_probe.hip — calibrates rocprofv3's FETCH_SIZE on gfx950 for the access shapes of the
// engine's gather kernels (MI355X_MICROARCH.md establishes FETCH_SIZE = half
// the bytes only for wide coalesced streaming reads).  Measurement tool, not part of the engine.
//
// Every kernel reads a known set of addresses in a 4 GiB buffer (far past the 256 MiB Infinity
// Cache, so every line comes from HBM once) and stores nothing (a never-true guard keeps the loads):
//   k_stream<W>      : coalesced W bytes per lane over the first STREAM_BYTES       (W = 8, 16)
//   k_gather<W, G>   : groups of G consecutive lanes read G*W contiguous bytes at a pseudo-random
//                      G*W-aligned address (G = 1: every lane its own line)       (W = 4, 8, 16)
// The host replays the same address hash and prints, per kernel, the useful bytes and the
// distinct 64-B and 128-B lines touched; rocprofv3 --pmc FETCH_SIZE over this binary gives the
// counted bytes, so counted / distinct lines says how a gather is tallied.
//
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_probe.hip -o tools/fetch_probe
//   rocprofv3 --pmc FETCH_SIZE -d out -o fp --output-format csv -- tools/fetch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

constexpr uint64_t BUF_BYTES = 4ull << 30;
constexpr uint64_t STREAM_BYTES = 1ull << 30;
constexpr uint64_t GROUPS = 1ull << 21;        // gather groups per kernel

__host__ __device__ inline uint64_t mix(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

template <int W> struct Vec;
template <> struct Vec<4> { typedef uint32_t T; };
template <> struct Vec<8> { typedef uint64_t T; };
template <> struct Vec<16> { typedef unsigned long long T __attribute__((ext_vector_type(2))); };

template <int W> __device__ inline uint64_t fold(typename Vec<W>::T x) { return (uint64_t)x; }
template <> __device__ inline uint64_t fold<16>(Vec<16>::T x) { return x.x ^ x.y; }

template <int W>
__global__ __launch_bounds__(256) void k_stream(const uint8_t *buf, uint64_t *sink)
{
    typedef typename Vec<W>::T T;
    const T *p = reinterpret_cast<const T *>(buf);
    const uint64_t n = STREAM_BYTES / W, stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc = acc * 31 + fold<W>(p[i]);
    if (acc == 0x0123456789abcdefull) sink[0] = acc;
}

template <int W, int G>
__global__ __launch_bounds__(256) void k_gather(const uint8_t *buf, uint64_t *sink, uint64_t salt)
{
    typedef typename Vec<W>::T T;
    const uint64_t chunks = BUF_BYTES / (uint64_t)(W * G);
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t t = tid; t < GROUPS * G; t += stride) {
        const uint64_t g = t / G, k = t % G;
        const uint64_t c = mix(g ^ salt) % chunks;
        // (a multiply, not a xor: with 4-B loads the guard's upper half must stay reachable)
        acc = acc * 31 + fold<W>(*reinterpret_cast<const T *>(buf + c * (uint64_t)(W * G) + k * W));
    }
    if (acc == 0x0123456789abcdefull) sink[0] = acc;
}

static void lines(int W, int G, uint64_t salt, uint64_t &l64, uint64_t &l128)
{
    std::vector<uint64_t> a(GROUPS), b(GROUPS);
    const uint64_t chunks = BUF_BYTES / (uint64_t)(W * G);
    for (uint64_t g = 0; g < GROUPS; ++g) {
        const uint64_t base = (mix(g ^ salt) % chunks) * (uint64_t)(W * G);
        a[g] = base / 64; b[g] = base / 128;          // a chunk of <= 64 B lies in one 64-B line
    }
    std::sort(a.begin(), a.end()); std::sort(b.begin(), b.end());
    l64 = std::unique(a.begin(), a.end()) - a.begin();
    l128 = std::unique(b.begin(), b.end()) - b.begin();
    if (W * G == 128) l64 *= 2;                       // a 128-B chunk covers two 64-B lines
}

template <int W, int G> static void gather(const uint8_t *buf, uint64_t *sink, int cus, uint64_t salt)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_gather<W, G>), dim3(cus * 8), dim3(256), 0, 0, buf, sink, salt);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint64_t l64 = 0, l128 = 0;
    lines(W, G, salt, l64, l128);
    printf("{\"kernel\": \"k_gather<%d, %d>\", \"useful_bytes\": %llu, \"lines64\": %llu, \"lines128\": %llu, \"ms\": %.4f}\n",
           W, G, (unsigned long long)(GROUPS * G * W), (unsigned long long)l64, (unsigned long long)l128, ms);
}

int main()
{
    uint8_t *buf = nullptr;
    uint64_t *sink = nullptr;
    if (hipMalloc(&buf, BUF_BYTES) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 1, BUF_BYTES);
    hipDeviceSynchronize();
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipLaunchKernelGGL((k_stream<16>), dim3(cus * 8), dim3(256), 0, 0, buf, sink);
    hipLaunchKernelGGL((k_stream<8>), dim3(cus * 8), dim3(256), 0, 0, buf, sink);
    hipDeviceSynchronize();
    printf("{\"kernel\": \"k_stream<16>\", \"useful_bytes\": %llu}\n", (unsigned long long)STREAM_BYTES);
    printf("{\"kernel\": \"k_stream<8>\", \"useful_bytes\": %llu}\n", (unsigned long long)STREAM_BYTES);
    // distinct salts: no kernel finds another's lines in a cache
    gather<4, 1>(buf, sink, cus, 11);
    gather<8, 1>(buf, sink, cus, 12);
    gather<16, 1>(buf, sink, cus, 13);
    gather<8, 8>(buf, sink, cus, 14);      // 64 B per group
    gather<8, 16>(buf, sink, cus, 15);     // 128 B per group
    gather<16, 8>(buf, sink, cus, 16);     // 128 B per group, 16 B per lane
    hipFree(buf); hipFree(sink);
    return 0;
}

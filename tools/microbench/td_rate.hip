// Vector-memory data-path microbenchmark (gfx950): throughput of lane-divergent 16-B and 4-B
// loads from an L2-resident buffer, by the number of active lanes per wave instruction.
// Does the cost of a wave's load instruction follow its instruction count or its active lanes'
// bytes? (the C5 walk's TD is 92% busy.)
// build: hipcc --offload-arch=gfx950 -O3 td_rate.hip -o td_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int kWide>
__global__ void __launch_bounds__(256) k(const uint4* __restrict__ buf, uint32_t mask, uint32_t* out, int iters,
                                         uint32_t active) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t i0 = (blockIdx.x * 256u + threadIdx.x) * 2654435761u, i1 = i0 ^ 0x9e3779b9u, i2 = i0 + 12345u,
             i3 = i0 * 7u + 1u;
    uint32_t acc = 0;
    if (lane < active) {
        for (int it = 0; it < iters; ++it) {
            if (kWide) {
                const uint4 a = buf[i0 & mask], b = buf[i1 & mask], c = buf[i2 & mask], d = buf[i3 & mask];
                i0 = i0 * 1664525u + 1013904223u + a.x;
                i1 = i1 * 1664525u + 1013904223u + b.y;
                i2 = i2 * 1664525u + 1013904223u + c.z;
                i3 = i3 * 1664525u + 1013904223u + d.w;
            } else {
                const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
                const uint32_t a = b32[i0 & (4u * mask + 3u)], b = b32[i1 & (4u * mask + 3u)],
                               c = b32[i2 & (4u * mask + 3u)], d = b32[i3 & (4u * mask + 3u)];
                i0 = i0 * 1664525u + 1013904223u + a;
                i1 = i1 * 1664525u + 1013904223u + b;
                i2 = i2 * 1664525u + 1013904223u + c;
                i3 = i3 * 1664525u + 1013904223u + d;
            }
        }
        acc = i0 ^ i1 ^ i2 ^ i3;
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

// Where the divergent loads' limit sits: the same 16-B loads from an L1-sized buffer, and with
// 8 lanes reading the 8 adjacent 16-B slots of one 128-B line (the cooperative leaf batches'
// pattern) instead of 8 lines.
template <int kGroup>
__global__ void __launch_bounds__(256) kg(const uint4* __restrict__ buf, uint32_t mask, uint32_t* out, int iters) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = (blockIdx.x * 256u + threadIdx.x) / kGroup, j = lane % kGroup;
    uint32_t i0 = g * 2654435761u, i1 = i0 ^ 0x9e3779b9u, i2 = i0 + 12345u, i3 = i0 * 7u + 1u;
    for (int it = 0; it < iters; ++it) {
        const uint32_t m = mask & ~(uint32_t)(kGroup - 1);
        const uint4 a = buf[(i0 & m) + j], b = buf[(i1 & m) + j], c = buf[(i2 & m) + j], d = buf[(i3 & m) + j];
        i0 = i0 * 1664525u + 1013904223u + a.x;
        i1 = i1 * 1664525u + 1013904223u + b.y;
        i2 = i2 * 1664525u + 1013904223u + c.z;
        i3 = i3 * 1664525u + 1013904223u + d.w;
    }
    out[blockIdx.x * 256u + threadIdx.x] = i0 ^ i1 ^ i2 ^ i3;
}

int main() {
    const uint32_t n = 1u << 17;  // 2 MiB of uint4: L2-resident
    uint4* buf;
    uint32_t* out;
    (void)hipMalloc(&buf, n * sizeof(uint4));
    (void)hipMemset(buf, 1, n * sizeof(uint4));
    const int blocks = 256 * 8;
    (void)hipMalloc(&out, blocks * 256 * 4);
    const int iters = 2000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int wide = 1; wide >= 0; --wide) {
        for (uint32_t active : {64u, 32u, 16u, 8u, 4u, 1u}) {
            float ms = 0.f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                if (wide) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, buf, n - 1u, out, iters, active);
                else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, buf, n - 1u, out, iters, active);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double waves = blocks * 4.0, winstr = waves * iters * 4.0, lanes = winstr * active;
            printf("%s loads, %2u active lanes: %8.3f ms  %7.1f G wave-instr/s  %8.1f G lane-loads/s  %7.1f GB/s\n",
                   wide ? "16-B" : " 4-B", active, ms, winstr / ms / 1e6, lanes / ms / 1e6,
                   lanes * (wide ? 16.0 : 4.0) / ms / 1e6);
        }
    }
    for (uint32_t words : {1u << 17, 1u << 10}) {  // 2 MiB (L2) or 16 KiB (L1) of uint4
        for (int group : {1, 8}) {
            float ms = 0.f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                if (group == 1) hipLaunchKernelGGL(kg<1>, dim3(blocks), dim3(256), 0, 0, buf, words - 1u, out, iters);
                else hipLaunchKernelGGL(kg<8>, dim3(blocks), dim3(256), 0, 0, buf, words - 1u, out, iters);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double lanes = blocks * 4.0 * iters * 4.0 * 64.0;
            printf("16-B loads, %6u KiB buffer, %d lane(s) per 128-B line: %8.3f ms  %8.1f G lane-loads/s  %8.1f G lines/s\n",
                   words / 64u, group, ms, lanes / ms / 1e6, lanes / group / ms / 1e6);
        }
    }
    return 0;
}

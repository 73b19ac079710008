// VALU issue-rate microbenchmark: v_mul_f32 vs v_pk_mul_f32 (gfx950).
// One block of 256 threads per CU x 8, 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int PK>
__global__ void k(float* out, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float s = 1.0001f;
    for (int i = 0; i < iters; ++i) {
        if (PK) {
            asm volatile(
                "v_pk_mul_f32 %0, %0, %8\n v_pk_mul_f32 %2, %2, %8\n v_pk_mul_f32 %4, %4, %8\n v_pk_mul_f32 %6, %6, %8\n"
                "v_pk_mul_f32 %0, %0, %8\n v_pk_mul_f32 %2, %2, %8\n v_pk_mul_f32 %4, %4, %8\n v_pk_mul_f32 %6, %6, %8\n"
                : "+v"(*(double*)&a0), "+v"(a1), "+v"(*(double*)&a2), "+v"(a3), "+v"(*(double*)&a4), "+v"(a5),
                  "+v"(*(double*)&a6), "+v"(a7)
                : "v"((double)0));
        } else {
            asm volatile(
                "v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n"
                "v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(s));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 2048 * 4);
    int iters = 20000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int blocks_per_cu : {1, 4, 8}) {
        int blocks = 256 * blocks_per_cu;
        for (int rep = 0; rep < 2; ++rep) {
            float ms[2];
            for (int pk = 0; pk < 2; ++pk) {
                (void)hipEventRecord(e0);
                if (pk) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
                else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms[pk], e0, e1);
            }
            double instr = (double)blocks * 4 * iters * 8;  // wave-instructions
            printf("blocks/CU %d: v_mul_f32 %.3f ms (%.1f G wave-instr/s)  v_pk_mul_f32 %.3f ms (%.1f G wave-instr/s)\n",
                   blocks_per_cu, ms[0], instr / ms[0] / 1e6, ms[1], instr / ms[1] / 1e6);
        }
    }
    return 0;
}
